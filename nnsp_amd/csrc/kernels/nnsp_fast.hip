// nnsp_fast.hip -- split NN path for nets with exactly one LSTM layer (all
// three reference nets: fc -> lstm -> fc -> fc -> fc).
//
// NeuralNetClass_exe (neural_nets.c:44-168) is recurrent only through the LSTM
// state; the layers before the LSTM and the LSTM's input half of every gate
// (rc_Krows_8x16's first affine, affine.c:377-384) depend on the frame's
// context alone.  So a chunk runs as
//   proj_kernel  : every (stream, NN step) row in parallel -- prefix FC
//                  layers + Wx.x -> exact int32 gate partial sums gx;
//                  16-row MFMA tiles = 16 consecutive steps of one stream (their
//                  context windows overlap: 36 feature frames feed 16 rows)
//   recur_kernel : per 16-stream tile, the steps in order -- Wh.h + gx, gate
//                  epilogue (shift_64b, bias, clamp/wrap, sigmoid/tanh), cell
//                  and hidden update (lstm.c:106-115, h after all groups: T6),
//                  the FC layers after the LSTM, post-processing, triggers.
// All weights of each kernel are staged once per workgroup into LDS as MFMA
// A-fragments.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nnsp_dev.h"
#include "nnsp_kabi.h"
#include "nnsp_nn.h"

using namespace nnsp;

#define P_ASTRIDE 264   // int16 per row of a proj activation buffer
#define P_UNION 1440    // 36 frames x 40 features (int16)
#define R_STRIDE 136    // int16 per row of recur h / activation buffers
#define R_CW 128        // int32 per row of the c buffer

// per-row epilogue constants, staged into LDS (global loads in the per-step
// epilogue put an L2 round trip on the recurrence's critical path).  bterm is
// the bias term affine_Krows_8x16 adds before the output shift (affine.c:190-217):
// b << (qbit_s - qb) (or >>), 64-bit for acc64, wrapping int32 for acc32.
struct EpRow {
    int32_t wsum, wsum_r;
    int64_t bterm;
};

__device__ __forceinline__ void stage_ep(EpRow* ep, const NnImage& img, int lo, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int row = lo + i;
        int li = 0;
        while (li + 1 < img.nl && img.L[li + 1].ep_off <= row) ++li;
        const NnLayer& Ly = img.L[li];
        const int16_t b = img.bias[row];
        int64_t bt = 0;
        if (Ly.has_bias) {
            if (img.acc32)
                bt = Ly.bias_sh >= 0 ? wshl(b, Ly.bias_sh) : ((int32_t)b >> -Ly.bias_sh);
            else
                bt = Ly.bias_sh >= 0 ? (int64_t)((uint64_t)(int64_t)b << Ly.bias_sh) : ((int64_t)b >> -Ly.bias_sh);
        }
        ep[i] = EpRow{img.wsum[row], img.wsum_r[row], bt};
    }
}

// affine_Krows_8x16 output stage with the bias term already folded in:
// shift_64b + clamp (acc64) or shift_32b (acc32).  rsh/lsh = the layer's
// output shift split by sign (lsh > 0 never happens for the reference nets).
template <bool ACC32>
__device__ __forceinline__ int32_t ep_shift(int64_t pre, int rsh, int lsh) {
    if (ACC32) {
        const int32_t v = (int32_t)pre;
        return __builtin_expect(lsh > 0, 0) ? shift32(v, lsh) : (v >> rsh);
    }
    return sat32(__builtin_expect(lsh > 0, 0) ? shift64(pre, lsh) : (pre >> rsh));
}

__host__ __device__ inline size_t ep_bytes(int n) { return ((size_t)n * sizeof(EpRow) + 15) & ~(size_t)15; }

struct ProjWave {
    int16_t uni[P_UNION + 32];
    int16_t act[2][16][P_ASTRIDE];
};

__device__ __forceinline__ void stage_weights(uint8_t* dst, const uint8_t* src, int bytes) {
    const int4* s = reinterpret_cast<const int4*>(src);
    int4* d = reinterpret_cast<int4*>(dst);
    for (int i = threadIdx.x; i < bytes / 16; i += blockDim.x) d[i] = s[i];
}

// One FC layer on a 16-row tile: B from an LDS buffer (row stride in_stride),
// A fragments from LDS, output to an LDS buffer (row stride out_stride).
__device__ __forceinline__ void fc_tile(const NnImage& img, const NnLayer& Ly, const uint8_t* A,
                                        const EpRow* ep, const int16_t* in, int in_stride, int16_t* out,
                                        int out_stride, const int16_t* tt, int lane) {
    v4i bh[4], bl[4];
    load_b<4>(in, in_stride, Ly.nkt, lane, bh, bl);
    const int sc = lane & 15, q = lane >> 4;
    for (int rt = 0; rt < Ly.nrt; ++rt) {
        v4i ah = {0, 0, 0, 0}, al = {0, 0, 0, 0};
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
            if (kt < Ly.nkt) {
                const v4i w = *reinterpret_cast<const v4i*>(A + (size_t)(rt * Ly.nkt + kt) * 1024 + 16 * lane);
                ah = mfma8(w, bh[kt], ah);
                al = mfma8(w, bl[kt], al);
            }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = 16 * rt + 4 * q + i;
            if (row >= Ly.rows) continue;
            const EpRow& er = ep[row];
            const int32_t sum = (ah[i] << 8) + al[i] + er.wsum;
            const int32_t v = img.acc32 ? shift32(wadd(sum, (int32_t)er.bterm), Ly.out_sh)
                                        : sat32(shift64((int64_t)sum + er.bterm, Ly.out_sh));
            if (Ly.act == ACT_LINEAR)
                reinterpret_cast<int32_t*>(out + sc * out_stride)[row] = v;
            else
                out[sc * out_stride + row] = act16(Ly.act, v, tt);
        }
    }
}

// ---------------------------------------------------------------------------
// proj_kernel
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void proj_kernel(NnImage img, FastRun r) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* W = smem;                                           // staged A fragments
    int16_t* tt = reinterpret_cast<int16_t*>(smem + r.a_lds_bytes);
    EpRow* ep = reinterpret_cast<EpRow*>(smem + r.a_lds_bytes + 768);
    ProjWave* pw = reinterpret_cast<ProjWave*>(smem + r.a_lds_bytes + 768 + ep_bytes(r.ep_n));
    stage_weights(W, img.A + r.a_off, r.a_lds_bytes);
    stage_ep(ep, img, r.ep_lo, r.ep_n);
    for (int i = threadIdx.x; i < 384; i += blockDim.x) tt[i] = nnsp_tbl_tanh[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    ProjWave& P = pw[wv];
    const int sc = lane & 15, q = lane >> 4;
    const NnLayer& LL = img.L[r.li];
    const int wsteps = r.seg_len > 0 ? min(r.nstep_max, (r.seg_len + 1) / 2) : r.nstep_max;
    const int ntps = (wsteps + 15) / 16;
    const int nrow = r.list ? r.n_list : r.S;
    const long long ntiles = (long long)nrow * ntps;
    const int rows = LL.rows;
    for (long long tile = (long long)blockIdx.x * (blockDim.x >> 6) + wv; tile < ntiles;
         tile += (long long)gridDim.x * (blockDim.x >> 6)) {
        const int i_row = (int)(tile / ntps), j0 = 16 * (int)(tile - (long long)i_row * ntps);
        const int s = r.list ? r.list[i_row] : i_row;
        const int b = r.seg_begin ? r.seg_begin[s] : 0;   // segment: frames b..e-1
        const int L = (r.seg_len > 0 ? min(r.T, b + r.seg_len) : r.T) - b;
        const int phase = 1 - reinterpret_cast<const NnPost*>(r.post)[s].slides;
        const int t0 = 2 * j0 + phase;            // segment-relative NN frame of row 0
        if (t0 >= L) continue;                    // wave-uniform
        // ---- union of the 16 context windows: V[t0 .. t0+35], V = prev5 ++ feats[b..T)
        for (int c = lane; c < 180; c += 64) {
            const int fr = c / 5, part = c - 5 * fr, idx = t0 + fr;
            int4 v = make_int4(0, 0, 0, 0);
            if (idx < 5)
                v = *reinterpret_cast<const int4*>(r.prev5 + ((size_t)s * 5 + idx) * 40 + 8 * part);
            else if (idx - 5 < L)
                v = *reinterpret_cast<const int4*>(r.feats + ((size_t)s * r.T + b + idx - 5) * 40 + 8 * part);
            *reinterpret_cast<int4*>(&P.uni[8 * c]) = v;
        }
        wave_lds_sync();
        // ---- prefix FC layers (row p's context = uni[80p .. 80p+239])
        const int16_t* in = P.uni;
        int in_stride = 80;
        for (int i = 0; i < r.li; ++i) {
            const NnLayer& Ly = img.L[i];
            int16_t* out = &P.act[i & 1][0][0];
            fc_tile(img, Ly, W + (Ly.a_off - r.a_off), ep + (Ly.ep_off - r.ep_lo), in, in_stride, out, P_ASTRIDE,
                    tt, lane);
            wave_lds_sync();
            in = out;
            in_stride = P_ASTRIDE;
        }
        // ---- LSTM input half: gx = sum_k Wx[row][k] x[k] (exact, before shift_64b)
        {
            v4i bh[4], bl[4];
            load_b<4>(in, in_stride, LL.nkt, lane, bh, bl);
            const uint8_t* A = W + (LL.a_off - r.a_off);
            const int j = j0 + sc;
            const bool act = j < r.nstep_max && 2 * j + phase < L;
            int32_t* dst = r.gx + ((size_t)s * r.nstep_max + j) * rows + 4 * q;
            for (int rt = 0; rt < LL.nrt; ++rt) {
                v4i ah = {0, 0, 0, 0}, al = {0, 0, 0, 0};
#pragma unroll
                for (int kt = 0; kt < 4; ++kt)
                    if (kt < LL.nkt) {
                        const v4i w = *reinterpret_cast<const v4i*>(A + (size_t)(rt * LL.nkt + kt) * 1024 + 16 * lane);
                        ah = mfma8(w, bh[kt], ah);
                        al = mfma8(w, bl[kt], al);
                    }
                const EpRow* er = ep + (LL.ep_off - r.ep_lo) + 16 * rt + 4 * q;
                int4 o;
                o.x = (ah[0] << 8) + al[0] + er[0].wsum;
                o.y = (ah[1] << 8) + al[1] + er[1].wsum;
                o.z = (ah[2] << 8) + al[2] + er[2].wsum;
                o.w = (ah[3] << 8) + al[3] + er[3].wsum;
                if (act) *reinterpret_cast<int4*>(dst + 16 * rt) = o;
            }
        }
        wave_lds_sync();
    }
}

// ---------------------------------------------------------------------------
// recur_kernel: one 16-stream tile per RW waves, TPW tiles per workgroup;
// weights and epilogue constants staged once per workgroup.
//   waves 0..RG-1 ("LSTM waves"): step j -- Wh.h + gx, gate epilogue, cell and
//                 hidden update; LSTM row tiles dealt round-robin;
//   wave  RG      ("tail wave"):  step j-1 -- the FC layers after the LSTM,
//                 post-processing, trigger / logits / outputs stores.
// Nothing recurrent depends on the tail, so it runs one step behind the LSTM
// waves with a single workgroup barrier per step.  h is double-buffered: step
// j reads h[cur] and writes h[cur^1]; the tail reads h[cur] (step j-1's
// result) in the same iteration; step j+1 overwrites h[cur] only after the
// next barrier, which the tail reaches once it is done with it.
// ---------------------------------------------------------------------------
#define RG 4
#define RW (RG + 1)

struct RecTile {
    int16_t h[2][16][R_STRIDE];     // LSTM h, ping-pong across steps
    int16_t act[2][16][R_STRIDE];   // tail wave: FC activations, ping-pong across layers
    int32_t c[16][R_CW];
    int32_t phase[16];
    int32_t nst[16];    // NN steps of each stream's segment
    int32_t beg[16];    // segment start frame
    int32_t end[16];    // segment end frame (exclusive)
};

template <int RPW, bool ACC32>   // RPW: LSTM row tiles per wave = ceil(nrt / RG)
__global__ __launch_bounds__(64 * RW * 2) void recur_kernel(NnImage img, FastRun r) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* W = smem;
    int16_t* tt = reinterpret_cast<int16_t*>(smem + r.a_lds_bytes);
    EpRow* ep = reinterpret_cast<EpRow*>(smem + r.a_lds_bytes + 768);
    RecTile* tiles = reinterpret_cast<RecTile*>(smem + r.a_lds_bytes + 768 + ep_bytes(r.ep_n));
    stage_weights(W, img.A + r.a_off, r.a_lds_bytes);
    stage_ep(ep, img, r.ep_lo, r.ep_n);
    for (int i = threadIdx.x; i < 384; i += blockDim.x) tt[i] = nnsp_tbl_tanh[i];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int tpw = blockDim.x / (64 * RW);
    const int tl = wv / RW, g = wv - tl * RW;   // tile in workgroup, wave in tile
    const bool tail = g == RG;
    RecTile& R = tiles[tl];
    const int sc = lane & 15, q = lane >> 4;
    // tile = 16 consecutive entries of the stream list (identity when list == NULL)
    const int nrow = r.list ? r.n_list : r.S;
    const int i0 = (blockIdx.x * tpw + tl) * 16;
    auto sid = [&](int i) { return r.list ? r.list[i] : i; };
    const bool valid = i0 + sc < nrow;
    const int s = valid ? sid(i0 + sc) : 0;
    const NnLayer& LL = img.L[r.li];
    const int N = LL.N, rows = LL.rows, nrt = LL.nrt, nkt_r = LL.nkt_r;
    const int xs_sh = LL.xs_sh, rsh = LL.out_sh < 0 ? -LL.out_sh : 0, lsh = LL.out_sh > 0 ? LL.out_sh : 0;
    for (int idx = g * 64 + lane; idx < 16 * N; idx += 64 * RW) {
        const int st = idx / N, u = idx - st * N;
        const bool ok = i0 + st < nrow;
        const int gs = ok ? sid(i0 + st) : 0;
        R.h[0][st][u] = ok ? r.h[(size_t)gs * NN_MAX_W + u] : (int16_t)0;
        R.c[st][u] = ok ? r.c[(size_t)gs * NN_MAX_W + u] : 0;
    }
    const int T = r.T;
    PostState ps = {};
    if (tail && lane < 16) {
        const int b = valid && r.seg_begin ? r.seg_begin[s] : 0;
        const int e = r.seg_len > 0 ? min(T, b + r.seg_len) : T;
        if (valid) ps = reinterpret_cast<const PostState*>(r.post)[s];
        const int ph = valid ? 1 - ps.slides : 0;
        R.phase[lane] = ph;
        R.beg[lane] = b;
        R.end[lane] = e;
        R.nst[lane] = valid && e - b - ph > 0 ? (e - b - ph + 1) / 2 : 0;
    }
    __syncthreads();
    const int phase = R.phase[sc];
    const int b = R.beg[sc];
    const int e = R.end[sc];   // segment: frames b..e-1
    int nsteps = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) nsteps = max(nsteps, R.nst[i]);
    if (tail && lane < 16 && valid && phase == 1 && b < e) {   // frame b: no NN, trigger carried
        if (r.trig) r.trig[(size_t)s * T + b] = ps.trigger;
        if (r.out3)
            for (int o = 0; o < 3; ++o) r.out3[((size_t)s * T + b) * 3 + o] = ps.outputs[o];
    }
    const uint8_t* Ar = W;   // LSTM recurrent fragments lead the staged region
    const EpRow* epl = ep + (LL.ep_off - r.ep_lo);
    v4i gxv[RPW];
    auto load_gx = [&](int jj) {
        const bool ok = valid && b + 2 * jj + phase < e;
        const int32_t* gsrc = r.gx + ((size_t)(ok ? s : 0) * r.nstep_max + (ok ? jj : 0)) * rows + 4 * q;
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            const int rt = g + RG * k;
            if (rt < nrt) gxv[k] = *reinterpret_cast<const v4i*>(gsrc + 16 * rt);
        }
    };
    if (!tail) load_gx(0);
    long long* clk = (r.dbg_clk && blockIdx.x == 0 && tl == 0 && (g == 0 || tail)) ? r.dbg_clk + (tail ? 4 : 0)
                                                                                     : nullptr;
#define PROBE(k) \
    if (clk && j < 64) clk[j * 8 + (k)] = (long long)__builtin_amdgcn_s_memtime()
    int cur = 0;
    for (int j = 0; j <= nsteps; ++j) {
        PROBE(0);
        if (!tail) {
            if (j < nsteps) {
                // ---- LSTM step j (lstm.c:48-124): row tile = 4 units x gates i, j, f, o
                const int t = b + 2 * j + phase;
                const bool active = valid && t < e;
                v4i bh[2], bl[2];
                load_b<2>(&R.h[cur][0][0], R_STRIDE, nkt_r, lane, bh, bl);
#pragma unroll
                for (int k = 0; k < RPW; ++k) {
                    const int rt = g + RG * k;
                    if (rt < nrt) {
                        v4i hh = {0, 0, 0, 0}, hl = {0, 0, 0, 0};
#pragma unroll
                        for (int kt = 0; kt < 2; ++kt)
                            if (kt < nkt_r) {
                                const v4i w = *reinterpret_cast<const v4i*>(Ar + (size_t)(rt * nkt_r + kt) * 1024 + 16 * lane);
                                hh = mfma8(w, bh[kt], hh);
                                hl = mfma8(w, bl[kt], hl);
                            }
                        const int u = 4 * rt + q;
                        if (u < N) {
                            int16_t gt[4];
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                const EpRow& er = epl[16 * rt + 4 * q + i];
                                const int32_t sx = gxv[k][i];
                                const int32_t sh = (hh[i] << 8) + hl[i] + er.wsum_r;
                                int64_t pre;
                                if (ACC32) {
                                    const int32_t x = __builtin_expect(xs_sh != 0, 0) ? shift32(sx, xs_sh) : sx;
                                    pre = wadd(wadd(x, sh), (int32_t)er.bterm);
                                } else {
                                    const int64_t x = __builtin_expect(xs_sh != 0, 0) ? shift64((int64_t)sx, xs_sh)
                                                                                      : (int64_t)sx;
                                    pre = x + sh + er.bterm;
                                }
                                const int32_t v = ep_shift<ACC32>(pre, rsh, lsh);
                                gt[i] = i == 1 ? tanh_q15(v, tt) : sigmoid_q15(v, tt);
                            }
                            const int32_t c_old = R.c[sc][u];
                            const int32_t c_new = sat32(((int64_t)gt[0] * gt[1] + (int64_t)gt[2] * c_old) >> 15);
                            const int16_t hv = sat16(((int32_t)tanh_q15(c_new, tt) * gt[3]) >> 15);
                            if (active) R.c[sc][u] = c_new;
                            R.h[cur ^ 1][sc][u] = active ? hv : R.h[cur][sc][u];   // h after all groups (T6)
                        }
                    }
                }
                if (j + 1 < nsteps) load_gx(j + 1);
            }
        } else if (j > 0) {
            // ---- tail: step j-1's FC layers after the LSTM, outputs, post-processing
            const int jj = j - 1;
            const int t = b + 2 * jj + phase;
            const bool active = valid && t < e;
            const int16_t* in = &R.h[cur][0][0];
            int ab = 0;
            for (int i = r.li + 1; i < img.nl; ++i) {
                const NnLayer& Ly = img.L[i];
                const uint8_t* A = W + (Ly.a_off - r.a_off);
                const EpRow* epi = ep + (Ly.ep_off - r.ep_lo);
                const int nkt = Ly.nkt, lrt = Ly.nrt, lrows = Ly.rows, act = Ly.act;
                const int ors = Ly.out_sh < 0 ? -Ly.out_sh : 0, ols = Ly.out_sh > 0 ? Ly.out_sh : 0;
                int16_t* out = &R.act[ab][0][0];
                v4i fh[2], fl[2];
                load_b<2>(in, R_STRIDE, nkt, lane, fh, fl);
                for (int rt = 0; rt < lrt; ++rt) {
                    v4i ah = {0, 0, 0, 0}, al = {0, 0, 0, 0};
#pragma unroll
                    for (int kt = 0; kt < 2; ++kt)
                        if (kt < nkt) {
                            const v4i w = *reinterpret_cast<const v4i*>(A + (size_t)(rt * nkt + kt) * 1024 + 16 * lane);
                            ah = mfma8(w, fh[kt], ah);
                            al = mfma8(w, fl[kt], al);
                        }
#pragma unroll
                    for (int x = 0; x < 4; ++x) {
                        const int row = 16 * rt + 4 * q + x;
                        if (row >= lrows) continue;
                        const EpRow& er = epi[row];
                        const int32_t sum = (ah[x] << 8) + al[x] + er.wsum;
                        const int64_t pre = ACC32 ? (int64_t)wadd(sum, (int32_t)er.bterm) : (int64_t)sum + er.bterm;
                        const int32_t v = ep_shift<ACC32>(pre, ors, ols);
                        if (act == ACT_LINEAR)
                            reinterpret_cast<int32_t*>(out + sc * R_STRIDE)[row] = v;
                        else
                            out[sc * R_STRIDE + row] = act16(act, v, tt);
                    }
                }
                wave_lds_sync();
                in = out;
                ab ^= 1;
            }
            // outputs and post-processing (nn_speech.c:92-124)
            const int16_t* fin = in + sc * R_STRIDE;
            const NnLayer& LO = img.L[img.nl - 1];
            const int nout = LO.N;
            const bool lin = LO.act == ACT_LINEAR;
            if (active && r.logits) {
                int32_t* dst = r.logits + ((size_t)s * T + t) * nout;
                for (int o = q; o < nout; o += 4)
                    dst[o] = lin ? reinterpret_cast<const int32_t*>(fin)[o] : (int32_t)fin[o];
            }
            if (lane < 16 && active) {
                const LogitRow lg = {fin, lin};
                post_proc(ps, img, lg);
                if (r.trig) {
                    r.trig[(size_t)s * T + t] = ps.trigger;
                    if (t + 1 < e) r.trig[(size_t)s * T + t + 1] = ps.trigger;
                }
                if (r.out3)
                    for (int f = t; f < min(t + 2, e); ++f)
                        for (int o = 0; o < 3; ++o) r.out3[((size_t)s * T + f) * 3 + o] = ps.outputs[o];
            }
        }
        PROBE(1);
        __syncthreads();
        PROBE(2);
        cur ^= 1;
    }
#undef PROBE
    // ---- state out: the last LSTM step (iteration nsteps-1) wrote the buffer that
    // became cur at iteration nsteps; the tail-only iteration flipped cur once more
    for (int idx = g * 64 + lane; idx < 16 * N; idx += 64 * RW) {
        const int st = idx / N, u = idx - st * N;
        if (i0 + st < nrow) {
            const int gs = sid(i0 + st);
            r.h[(size_t)gs * NN_MAX_W + u] = R.h[cur ^ 1][st][u];
            r.c[(size_t)gs * NN_MAX_W + u] = R.c[st][u];
        }
    }
    if (tail && lane < 16 && valid && b < e) {
        ps.slides = (int16_t)(ps.slides ^ ((e - b) & 1));
        reinterpret_cast<PostState*>(r.post)[s] = ps;
    }
}

extern "C" {

size_t nnspk_fast_lds_bytes(int which, int a_bytes, int units, int ep_rows) {
    // which 0: proj (units = waves); 1: recur (units = tiles per workgroup)
    const size_t base = (size_t)a_bytes + 768 + ep_bytes(ep_rows);
    if (which == 0) return base + (size_t)units * sizeof(ProjWave);
    return base + (size_t)units * sizeof(RecTile);
}

int nnspk_launch_proj(const NnImage* img, const FastRun* r, int blocks, void* stream) {
    const size_t lds = nnspk_fast_lds_bytes(0, r->a_lds_bytes, 4, r->ep_n);
    hipLaunchKernelGGL(proj_kernel, dim3(blocks), dim3(256), lds, (hipStream_t)stream, *img, *r);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

int nnspk_launch_recur(const NnImage* img, const FastRun* r, int tpw, void* stream) {
    const size_t lds = nnspk_fast_lds_bytes(1, r->a_lds_bytes, tpw, r->ep_n);
    const int nrow = r->list ? r->n_list : r->S;
    if (nrow <= 0) return 0;
    const int tiles = (nrow + 15) / 16;
    const int blocks = (tiles + tpw - 1) / tpw;
    const int rpw = (img->L[r->li].nrt + RG - 1) / RG;
    const dim3 grid(blocks), blk(64 * RW * tpw);
    const hipStream_t st = (hipStream_t)stream;
#define LAUNCH(R_)                                                                        \
    do {                                                                                  \
        if (img->acc32)                                                                   \
            hipLaunchKernelGGL((recur_kernel<R_, true>), grid, blk, lds, st, *img, *r);  \
        else                                                                              \
            hipLaunchKernelGGL((recur_kernel<R_, false>), grid, blk, lds, st, *img, *r); \
    } while (0)
    if (rpw <= 2)
        LAUNCH(2);
    else if (rpw <= 4)
        LAUNCH(4);
    else if (rpw <= 5)
        LAUNCH(5);
    else
        LAUNCH(8);
#undef LAUNCH
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

int nnspk_set_lds_limit(void) {
    // allow up to 160 KiB of dynamic LDS for the split kernels
    hipError_t e = hipFuncSetAttribute((const void*)proj_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int)e;
    const void* ks[8] = {(const void*)recur_kernel<2, false>, (const void*)recur_kernel<4, false>,
                         (const void*)recur_kernel<5, false>, (const void*)recur_kernel<8, false>,
                         (const void*)recur_kernel<2, true>,  (const void*)recur_kernel<4, true>,
                         (const void*)recur_kernel<5, true>,  (const void*)recur_kernel<8, true>};
    for (int i = 0; i < 8; ++i) {
        e = hipFuncSetAttribute(ks[i], hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return (int)e;
    }
    return 0;
}

}  // extern "C"
