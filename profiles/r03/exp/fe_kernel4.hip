// fe_kernel4: four frames per wave (measured slower, not built) -- kept as the
// record of the experiment in DESIGN.md 3.1 (round 3).  It was compiled into
// nnsp_kernels.hip after fe_kernel2 and launched from nnspk_launch_fe for the
// shipped build's batch and shared modes; parity tests passed with it.
// ---- four frames per wave (FE_MODE_BATCH / FE_MODE_SHARED, shipped build) --
// One wave runs four frames at a time, 16 lanes per frame.  Lane l of a frame
// holds 16 of its 256 complex values, so two radix-4 stages run inside the
// lane's registers and one LDS transpose replaces fe_kernel's three exchanges
// (its T1 / T3 are 16 permlane swaps per frame, each ~3 VALU issue slots):
//   stages 1-2  lane l = 4*d1 + d0, register r = 4*d3 + d2 (stage 1
//               butterflies over d3 for each d2, stage 2 over d2 for each d3)
//   transpose   position 16h + lo at slot 16h + (lo ^ h): the stores (16
//               lanes, 16 consecutive slots) and the loads (16 lanes, one
//               slot per 16-slot row, low nibbles all different) both
//               conflict-free
//   stages 3-4  lane l = 4*e3 + e2, register m = 4*d1 + d0
// The split, the power spectrum and the Mel MACs then run frame by frame on
// all 64 lanes as in fe_kernel (the same butterflies, split and MACs: the
// same bits), and the log10 / normalisation tail packs the four frames' 160
// (frame, bank) items into three 64-lane passes instead of four 40-lane ones.
// Per wave: four frame buffers of 256 complex -- the transpose, the cFFT
// output, the power spectrum in place, the Mel partial sums behind it.
#define FE4_XS 544   // dwords per frame buffer: 512 (256 complex) + 32 (frames 0 / 1 and 2 / 3 on opposite
                     // halves of the bank row for the transpose loads; the zero Mel slot at 512)
#define FE4_MS 384   // the frame's 64 Mel partial sums (int64) at dwords 384..511 (past the power spectrum)
#define FE4_WAVES 8

struct Fe4Tables {
    int2 tw1[3][64];     // stage 1: twiddles W^{(j+1)k} (cos, sin), k = 16*d2 + l
    int2 tw2[3][16];     // stage 2: k = 4*(4*d1 + d0) = 4l
    int4 split[256];     // per bin k: (A_re, A_im, B_re, norm word): FeTables.split; batch mode: mean of
                         // bank k < 40, stdR of bank k - 40 < 40
    uint32_t logp[128];  // log_tayler_coeff (value, slope) pairs
    uint4 win[16][4];    // lane l: window taps 2c, 2c+1 of c = 16r + l as int16 pairs, r = 4q + i in
                         // win[l][q ^ (l >> 2 & 3)].i (0 past tap 479; conflict-free b128 reads)
    uint2 mc[3][64];     // per lane segment: Mel coefficients as int16 pairs (FeTables.mc)
    uint32_t bank[40];   // bank b: its <= 3 lane segments (7 bits each; unused: 64, the zero slot)
};

template <class T4>
__device__ __forceinline__ T4 sel4(int i, T4 x0, T4 x1, T4 x2, T4 x3) {
    return i == 0 ? x0 : (i == 1 ? x1 : (i == 2 ? x2 : x3));
}

template <int MODE>
__global__ __launch_bounds__(64 * FE4_WAVES) __attribute__((amdgpu_waves_per_eu(4, 4))) void fe_kernel4(FeArgs a) {
    static_assert(MODE != FE_MODE_COLD, "the cold front end runs fe_kernel");
    constexpr bool shared = MODE == FE_MODE_SHARED;
    __shared__ __attribute__((aligned(16))) int32_t XB[FE4_WAVES][4 * FE4_XS];
    __shared__ __attribute__((aligned(16))) Fe4Tables TB;
    const unsigned nrow = a.n_list_dev ? (unsigned)*a.n_list_dev : (a.list ? (unsigned)a.n_list : (unsigned)a.S);
    const unsigned W = (unsigned)a.T;   // no segments (the host runs fe_kernel for those)
    const unsigned nfr = nrow * W;      // host guarantees < 2^31
    const unsigned nw = gridDim.x * FE4_WAVES;
    const unsigned per = ((nfr + nw - 1) / nw + 3) & ~3u;   // whole groups of four frames per wave
    if (blockIdx.x * FE4_WAVES * per >= nfr) return;   // no frame for this workgroup
    const int tid = threadIdx.x;
    for (int i = tid; i < 192; i += 64 * FE4_WAVES) {
        const int j = i / 64, k = i % 64;
        TB.tw1[j][k] = make_int2(nnsp_tbl_tw256[2 * (j + 1) * k], nnsp_tbl_tw256[2 * (j + 1) * k + 1]);
    }
    for (int k = tid; k < 256; k += 64 * FE4_WAVES) {
        int32_t nw32 = 0;
        if (shared)
            nw32 = fe_norm_word(a, k);
        else if (k < 80)
            nw32 = k < 40 ? a.mean[k] : a.stdR[k - 40];
        TB.split[k] = make_int4(nnsp_tbl_split[3 * k], nnsp_tbl_split[3 * k + 1], nnsp_tbl_split[3 * k + 2], nw32);
    }
    for (int i = tid; i < 48; i += 64 * FE4_WAVES) {
        const int j = i / 16, k = 4 * (i % 16);
        TB.tw2[j][i % 16] = make_int2(nnsp_tbl_tw256[2 * (j + 1) * k], nnsp_tbl_tw256[2 * (j + 1) * k + 1]);
    }
    for (int i = tid; i < 128; i += 64 * FE4_WAVES)
        TB.logp[i] = (uint32_t)(uint16_t)nnsp_tbl_log[2 * i] | ((uint32_t)(uint16_t)nnsp_tbl_log[2 * i + 1] << 16);
    for (int i = tid; i < 256; i += 64 * FE4_WAVES) {
        const int l = i / 16, r = i % 16, c = 16 * r + l;
        const uint32_t w = 2 * c < 480 ? ((uint32_t)(uint16_t)nnsp_tbl_window[2 * c] |
                                          ((uint32_t)(uint16_t)nnsp_tbl_window[2 * c + 1] << 16))
                                       : 0u;
        reinterpret_cast<uint32_t*>(&TB.win[l][(r >> 2) ^ ((l >> 2) & 3)])[r & 3] = w;
    }
    if (tid < 64) {
        const int* sg = nnsp_tbl_melseg + 4 * tid;
        const int mn = sg[2];
        uint32_t c[6];
        for (int i = 0; i < 6; ++i) {
            const int lo = 2 * i < mn ? nnsp_tbl_mel[sg[3] + 2 * i] : 0;
            const int hi = 2 * i + 1 < mn ? nnsp_tbl_mel[sg[3] + 2 * i + 1] : 0;
            c[i] = (uint32_t)(uint16_t)lo | ((uint32_t)(uint16_t)hi << 16);
        }
        for (int j = 0; j < 3; ++j) TB.mc[j][tid] = make_uint2(c[2 * j], c[2 * j + 1]);
    } else if (tid < 64 + 40) {
        const int b = tid - 64;
        uint32_t off = 0;
        int n = 0;
        for (int k = 0; k < 64; ++k)
            if (nnsp_tbl_melseg[4 * k] == b && n < FE_MEL_MAXSEG) off |= (uint32_t)k << (7 * n++);
        for (; n < FE_MEL_MAXSEG; ++n) off |= 64u << (7 * n);
        TB.bank[b] = off;
    }
    for (int i = tid; i < FE4_WAVES * 4; i += 64 * FE4_WAVES) {   // the zero Mel slots
        XB[i / 4][(i % 4) * FE4_XS + 512] = 0;
        XB[i / 4][(i % 4) * FE4_XS + 513] = 0;
    }
    __syncthreads();
    const int lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int fi = lane >> 4, l = lane & 15;   // FFT phase: the lane's frame in the group, its lane in the frame
    int32_t* Xw = XB[wv];
    int32_t* Xf = Xw + fi * FE4_XS;
    Tw3 tw3[4];                                // stage 3: k = 16*d0 (wave-uniform)
#pragma unroll
    for (int d0 = 0; d0 < 4; ++d0) tw3[d0] = load_tw3(16 * d0);
    const int mj0 = nnsp_tbl_melseg[4 * lane + 1];
    // tail items: pass p runs item lane + 64p = (frame, bank), packed with the
    // bank's segments: bits 0-20 segments (7 bits each), 21-26 bank, 27-29 frame (4: none)
    uint32_t titem[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        const int item = lane + 64 * p;
        const int b = item < 160 ? item % 40 : 0;
        titem[p] = TB.bank[b] | ((uint32_t)b << 21) | ((uint32_t)(item < 160 ? item / 40 : 4) << 27);
    }
    const unsigned wid = blockIdx.x * FE4_WAVES + (unsigned)wv;
    const unsigned fbeg = wid * per;
    const unsigned fend = fbeg + per < nfr ? fbeg + per : nfr;
    if (fbeg >= fend) return;
    auto row = [&](unsigned i) -> int {
        if (i >= nrow) return 0;   // past the list (frames of a group past fend): any in-range row
        if constexpr (shared) return (int)i;
        return a.list ? a.list[i] : (int)i;
    };
    // group cursor (wave-uniform): row ci, frame ck of the group's first frame
    unsigned ci = fbeg / W, ck = fbeg - (fbeg / W) * W;
    int cs = row(ci);
    struct Grp { int s[4], t[4]; unsigned n; };
    auto take = [&](Grp& G, unsigned f) {   // the group at frame f; leaves the cursor at f + 4
        G.n = fend - f < 4u ? fend - f : 4u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            G.s[k] = cs;
            G.t[k] = (int)ck;
            if (++ck == W) { ck = 0; ++ci; cs = row(ci); }
        }
    };
    auto fptr = [&](int s, int fidx) -> const int16_t* {   // input frame fidx of stream s (fe_kernel2, b = 0)
        if (fidx < 0) return a.tail + (size_t)s * (a.tail_stride ? (unsigned)a.tail_stride : 320u) + (fidx + 2) * 160;
        if constexpr (shared) return a.pcm + ((size_t)s * a.T + fidx) * 160;
        const int x = fidx - a.lookback;
        return x >= 0 ? a.pcm + ((size_t)s * a.T + x) * 160
                      : a.hist + ((size_t)s * a.hist_frames + a.hist_frames + x) * 160;
    };
    uint32_t raw[15];   // the lane's window samples 2c, 2c+1, c = 16r + l (r = 15: taps past 479, zero)
    auto issue = [&](const Grp& G) {
        const int s = sel4(fi, G.s[0], G.s[1], G.s[2], G.s[3]);
        const int t = sel4(fi, G.t[0], G.t[1], G.t[2], G.t[3]);
        const int lb = shared ? 0 : a.lookback;
        bool common = true;   // wave-uniform: every frame's window is 480 contiguous samples of the chunk
#pragma unroll
        for (int k = 0; k < 4; ++k) common = common && G.t[k] - 2 - lb >= 0;
        if (common) {
            const char* q = reinterpret_cast<const char*>(a.pcm + ((size_t)s * a.T + (t - 2 - lb)) * 160) + 4 * l;
#pragma unroll
            for (int r = 0; r < 15; ++r) raw[r] = *reinterpret_cast<const uint32_t*>(q + 64 * r);
            return;
        }
        const char* q0 = reinterpret_cast<const char*>(fptr(s, t - 2)) + 4 * l;
        const char* q1 = reinterpret_cast<const char*>(fptr(s, t - 1)) + 4 * l;
        const char* q2 = reinterpret_cast<const char*>(fptr(s, t)) + 4 * l;
#pragma unroll
        for (int r = 0; r < 15; ++r)
            raw[r] = *reinterpret_cast<const uint32_t*>(r < 5 ? q0 + 64 * r : (r < 10 ? q1 + 64 * (r - 5) : q2 + 64 * (r - 10)));
    };
    const unsigned ring0 = shared ? (unsigned)a.abs0 % (unsigned)a.ring : 0u;
    const unsigned nstride = shared ? (unsigned)a.S * (unsigned)a.ring * 40u : 0u;   // elements between rings
    Grp nx;
    take(nx, fbeg);
    issue(nx);
    for (unsigned f = fbeg; f < fend; f += 4) {
        const Grp G = nx;
        if (shared && a.hist_out) {   // the lane's frame's own 160 samples are raw[10..14]
            const int s = sel4(fi, G.s[0], G.s[1], G.s[2], G.s[3]);
            const int t = sel4(fi, G.t[0], G.t[1], G.t[2], G.t[3]);
            if ((unsigned)fi < G.n && t >= a.T - a.hist_frames) {
                int16_t* h = a.hist_out + ((size_t)s * a.hist_frames + (t - (a.T - a.hist_frames))) * 160 + 2 * l;
#pragma unroll
                for (int r = 10; r < 15; ++r) *reinterpret_cast<uint32_t*>(h + 32 * (r - 10)) = raw[r];
            }
        }
        // ---- window (spectrogram_module.c:103-119), Q30: register r = complex 16r + l
        int32_t v[16][2];
        {
            const int sw = (l >> 2) & 3;
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const uint4 w4 = TB.win[l][q4 ^ sw];
                const uint32_t wn[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int r = 4 * q4 + i;
                    if (r < 15) {
                        v[r][0] = (int32_t)(int16_t)(wn[i] & 0xffff) * (int32_t)(int16_t)(raw[r] & 0xffff);
                        v[r][1] = (int32_t)(int16_t)(wn[i] >> 16) * (int32_t)(int16_t)(raw[r] >> 16);
                    } else {
                        v[r][0] = 0;
                        v[r][1] = 0;
                    }
                }
            }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) asm volatile("" : "+v"(v[r][0]), "+v"(v[r][1]));
        if (f + 4 < fend) {   // the next group's samples (raw is free now)
            take(nx, f + 4);
            issue(nx);
        }
        // ---- cFFT stages 1-2 in registers (arm_radix4_butterfly_q31)
#pragma unroll
        for (int d2 = 0; d2 < 4; ++d2) {
            const int k = 16 * d2 + l;
            Tw3 t1;
            const int2 x = TB.tw1[0][k], y = TB.tw1[1][k], z = TB.tw1[2][k];
            t1.c1 = x.x; t1.s1 = x.y; t1.c2 = y.x; t1.s2 = y.y; t1.c3 = z.x; t1.s3 = z.y;
            bfly4<true>(v[d2][0], v[d2][1], v[4 + d2][0], v[4 + d2][1], v[8 + d2][0], v[8 + d2][1], v[12 + d2][0],
                        v[12 + d2][1], t1);
        }
        Tw3 tw2;
        {
            const int2 x = TB.tw2[0][l], y = TB.tw2[1][l], z = TB.tw2[2][l];
            tw2.c1 = x.x; tw2.s1 = x.y; tw2.c2 = y.x; tw2.s2 = y.y; tw2.c3 = z.x; tw2.s3 = z.y;
        }
#pragma unroll
        for (int e3 = 0; e3 < 4; ++e3)
            bfly4<false>(v[4 * e3][0], v[4 * e3][1], v[4 * e3 + 1][0], v[4 * e3 + 1][1], v[4 * e3 + 2][0],
                         v[4 * e3 + 2][1], v[4 * e3 + 3][0], v[4 * e3 + 3][1], tw2);
        // ---- transpose through LDS: position 16r + l out, 16l + m in
#pragma unroll
        for (int r = 0; r < 16; ++r) *reinterpret_cast<int2*>(Xf + 2 * (16 * r + (l ^ r))) = make_int2(v[r][0], v[r][1]);
        wave_lds_sync();
        int32_t w[16][2];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const int2 p = *reinterpret_cast<const int2*>(Xf + 2 * (16 * l + (m ^ l)));
            w[m][0] = p.x;
            w[m][1] = p.y;
        }
        // ---- stages 3-4
#pragma unroll
        for (int d0 = 0; d0 < 4; ++d0)
            bfly4<false>(w[d0][0], w[d0][1], w[4 + d0][0], w[4 + d0][1], w[8 + d0][0], w[8 + d0][1], w[12 + d0][0],
                         w[12 + d0][1], tw3[d0]);
#pragma unroll
        for (int e1 = 0; e1 < 4; ++e1) bfly4_last(&w[4 * e1][0]);
        wave_lds_sync();   // every lane's transpose loads before the bin stores
        // register 4*e1 + m is DIF position 16l + 4*e1 + m; its bin is rev8 of that (arm_bitreversal_32)
#pragma unroll
        for (int m = 0; m < 16; ++m)
            *reinterpret_cast<int2*>(Xf + 2 * rev8(16 * l + m)) = make_int2(w[m][0], w[m][1]);
        wave_lds_sync();
        // ---- split + power (arm_split_rfft_q31, spec2pspec_arm), frame by frame on all 64 lanes;
        //      the power spectrum P[k] overwrites the frame's buffer (dword k) once all its reads are done
        {
            const int4 cf0 = TB.split[lane + 1], cf1 = TB.split[lane + 65];
            int2 zk[4][2], zn[4][2], z0[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int32_t* X = Xw + g * FE4_XS;
                zk[g][0] = *reinterpret_cast<const int2*>(X + 2 * (lane + 1));
                zn[g][0] = *reinterpret_cast<const int2*>(X + 2 * (255 - lane));
                zk[g][1] = *reinterpret_cast<const int2*>(X + 2 * (lane + 65));
                zn[g][1] = *reinterpret_cast<const int2*>(X + 2 * (191 - lane));
                z0[g] = *reinterpret_cast<const int2*>(X);
            }
            wave_lds_sync();
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                int32_t* P = Xw + g * FE4_XS;
#pragma unroll
                for (int pr = 0; pr < 2; ++pr) {
                    const int4 cf = pr ? cf1 : cf0;
                    const int k = lane + 1 + 64 * pr;
                    int32_t re0, im0, re1, im1;
                    split_pair(zk[g][pr].x, zk[g][pr].y, zn[g][pr].x, zn[g][pr].y, cf.x, cf.y, cf.z, re0, im0, re1, im1);
                    P[k] = pspec_of(re0, im0);
                    P[256 - k] = pspec_of(re1, im1);
                }
                if (lane == 0) {   // DC and Nyquist: (p0 + p1) >> 1, (p0 - p1) >> 1
                    P[0] = pspec_of(wadd(z0[g].x, z0[g].y) >> 1, 0);
                    P[256] = pspec_of(wsub(z0[g].x, z0[g].y) >> 1, 0);
                }
            }
        }
        wave_lds_sync();
        // ---- Mel (melSpecProc.c:6-27): lane segments of <= 12 MACs, partial sums behind P
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            int32_t* P = Xw + g * FE4_XS;
            int64_t mac = 0;
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const uint2 c2 = TB.mc[j][lane];
                const uint32_t cc[2] = {c2.x, c2.y};
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int i = 2 * j + h;
                    mac = mad_i64_i32((int32_t)(int16_t)(cc[h] & 0xffff), P[mj0 + 2 * i], mac);
                    mac = mad_i64_i32((int32_t)cc[h] >> 16, P[mj0 + 2 * i + 1], mac);
                }
            }
            *reinterpret_cast<int64_t*>(P + FE4_MS + 2 * lane) = mac;
        }
        wave_lds_sync();
        // ---- log10 (fixlog10.c:53-61) and normalisation (feature_module.c:67-73) of the
        //      group's 160 (frame, bank) items in three passes
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const uint32_t ti = titem[p];
            const int g = (int)(ti >> 27);
            if ((unsigned)g < G.n) {   // (G.n <= 4)
                const int64_t* ms = reinterpret_cast<const int64_t*>(Xw + g * FE4_XS + FE4_MS);
                const int64_t mac = ms[ti & 127] + ms[(ti >> 7) & 127] + ms[(ti >> 14) & 127];
                const int32_t lg = log10_q15_lds(sat32(mac >> 15), TB.logp);
                const int s = sel4(g, G.s[0], G.s[1], G.s[2], G.s[3]);
                const int t = sel4(g, G.t[0], G.t[1], G.t[2], G.t[3]);
                const int b = (int)((ti >> 21) & 63);
                if constexpr (shared) {
                    unsigned slot = ring0 + (unsigned)t;   // (abs0 + t) % ring, t < T <= ring
                    if (slot >= (unsigned)a.ring) slot -= (unsigned)a.ring;
                    int16_t* r0 = a.nring[0] + (((unsigned)s * (unsigned)a.ring + slot) * 40u + (unsigned)b);
                    int16_t nv[3];
#pragma unroll
                    for (int n = 0; n < 3; ++n) {
                        const int32_t mn = TB.split[40 * n + b].w, sr = TB.split[120 + 40 * n + b].w;
                        nv[n] = fe_norm(lg, mn, sr, a.nshift[n], a.norm32);
                    }
                    r0[0] = nv[0];
                    r0[nstride] = nv[1];
                    r0[2 * (size_t)nstride] = nv[2];
                } else {
                    a.feats[((size_t)s * a.T + t) * 40 + b] =
                        fe_norm(lg, TB.split[b].w, TB.split[40 + b].w, a.norm_shift, a.norm32);
                }
            }
        }
        wave_lds_sync();   // the tail's loads before the next group's transpose stores
    }
}

