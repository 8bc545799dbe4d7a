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
                                        const int16_t* in, int in_stride, int16_t* out, int out_stride,
                                        const int16_t* tt, int lane) {
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
            const int32_t sum = (ah[i] << 8) + al[i] + img.wsum[Ly.ep_off + row];
            const int32_t v = affine_out(sum, img.bias[Ly.ep_off + row], Ly, img.acc32);
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
    ProjWave* pw = reinterpret_cast<ProjWave*>(smem + r.a_lds_bytes + 768);
    stage_weights(W, img.A + r.a_off, r.a_lds_bytes);
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
            fc_tile(img, Ly, W + (Ly.a_off - r.a_off), in, in_stride, out, P_ASTRIDE, tt, lane);
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
                int4 o;
                o.x = (ah[0] << 8) + al[0] + img.wsum[LL.ep_off + 16 * rt + 4 * q + 0];
                o.y = (ah[1] << 8) + al[1] + img.wsum[LL.ep_off + 16 * rt + 4 * q + 1];
                o.z = (ah[2] << 8) + al[2] + img.wsum[LL.ep_off + 16 * rt + 4 * q + 2];
                o.w = (ah[3] << 8) + al[3] + img.wsum[LL.ep_off + 16 * rt + 4 * q + 3];
                if (act) *reinterpret_cast<int4*>(dst + 16 * rt) = o;
            }
        }
        wave_lds_sync();
    }
}

// ---------------------------------------------------------------------------
// recur_kernel: one 16-stream tile per RG waves (row tiles dealt round-robin),
// TPW tiles per workgroup; weights staged once per workgroup.
// ---------------------------------------------------------------------------
#define RG 4

struct RecTile {
    int16_t h[2][16][R_STRIDE];     // LSTM h, ping-pong across steps
    int16_t act[2][16][R_STRIDE];   // FC activations, ping-pong across layers
    int32_t c[16][R_CW];
    int32_t phase[16];
    int32_t nst[16];    // NN steps of each stream's segment
    int32_t beg[16];    // segment start frame
    int32_t end[16];    // segment end frame (exclusive)
};

template <int RPW>   // LSTM row tiles per wave = ceil(nrt / RG)
__global__ __launch_bounds__(512) void recur_kernel(NnImage img, FastRun r) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* W = smem;
    int16_t* tt = reinterpret_cast<int16_t*>(smem + r.a_lds_bytes);
    RecTile* tiles = reinterpret_cast<RecTile*>(smem + r.a_lds_bytes + 768);
    stage_weights(W, img.A + r.a_off, r.a_lds_bytes);
    for (int i = threadIdx.x; i < 384; i += blockDim.x) tt[i] = nnsp_tbl_tanh[i];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int tpw = blockDim.x / (64 * RG);
    const int tl = wv / RG, g = wv - tl * RG;   // tile in workgroup, wave in tile
    RecTile& R = tiles[tl];
    const int sc = lane & 15, q = lane >> 4;
    // tile = 16 consecutive entries of the stream list (identity when list == NULL)
    const int nrow = r.list ? r.n_list : r.S;
    const int i0 = (blockIdx.x * tpw + tl) * 16;
    auto sid = [&](int i) { return r.list ? r.list[i] : i; };
    const bool valid = i0 + sc < nrow;
    const int s = valid ? sid(i0 + sc) : 0;
    const NnLayer& LL = img.L[r.li];
    const int N = LL.N, rows = LL.rows, nrt = LL.nrt;
    for (int idx = g * 64 + lane; idx < 16 * N; idx += 64 * RG) {
        const int st = idx / N, u = idx - st * N;
        const bool ok = i0 + st < nrow;
        const int gs = ok ? sid(i0 + st) : 0;
        R.h[0][st][u] = ok ? r.h[(size_t)gs * NN_MAX_W + u] : (int16_t)0;
        R.c[st][u] = ok ? r.c[(size_t)gs * NN_MAX_W + u] : 0;
    }
    const int T = r.T;
    PostState ps = {};
    if (g == 0 && lane < 16) {
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
    if (g == 0 && lane < 16 && valid && phase == 1 && b < e) {   // frame b: no NN, trigger carried
        if (r.trig) r.trig[(size_t)s * T + b] = ps.trigger;
        if (r.out3)
            for (int o = 0; o < 3; ++o) r.out3[((size_t)s * T + b) * 3 + o] = ps.outputs[o];
    }
    const uint8_t* Ar = W;   // LSTM recurrent fragments lead the staged region
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
    load_gx(0);
    int hb = 0;
    for (int j = 0; j < nsteps; ++j) {
        const int t = b + 2 * j + phase;
        const bool active = valid && t < e;
        v4i bh[2], bl[2];
        load_b<2>(&R.h[hb][0][0], R_STRIDE, LL.nkt_r, lane, bh, bl);
        // ---- LSTM (lstm.c:48-124): row tile = 4 units x gates i, j, f, o
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            const int rt = g + RG * k;
            if (rt < nrt) {
                v4i hh = {0, 0, 0, 0}, hl = {0, 0, 0, 0};
#pragma unroll
                for (int kt = 0; kt < 2; ++kt)
                    if (kt < LL.nkt_r) {
                        const v4i w = *reinterpret_cast<const v4i*>(Ar + (size_t)(rt * LL.nkt_r + kt) * 1024 + 16 * lane);
                        hh = mfma8(w, bh[kt], hh);
                        hl = mfma8(w, bl[kt], hl);
                    }
                const int u = 4 * rt + q;
                if (u < N) {
                    int16_t gt[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int row = 16 * rt + 4 * q + i;
                        const int32_t sx = gxv[k][i];
                        const int32_t sh = (hh[i] << 8) + hl[i] + img.wsum_r[LL.ep_off + row];
                        int64_t pre;
                        if (img.acc32)
                            pre = (int64_t)wadd(shift32(sx, LL.xs_sh), sh);
                        else
                            pre = shift64((int64_t)sx, LL.xs_sh) + (int64_t)sh;
                        const int32_t v = affine_out(pre, img.bias[LL.ep_off + row], LL, img.acc32);
                        gt[i] = i == 1 ? tanh_q15(v, tt) : sigmoid_q15(v, tt);
                    }
                    const int32_t c_old = R.c[sc][u];
                    const int32_t c_new = sat32(((int64_t)gt[0] * gt[1] + (int64_t)gt[2] * c_old) >> 15);
                    const int16_t hv = sat16(((int32_t)tanh_q15(c_new, tt) * gt[3]) >> 15);
                    if (active) R.c[sc][u] = c_new;
                    R.h[hb ^ 1][sc][u] = active ? hv : R.h[hb][sc][u];   // h after all groups (T6)
                }
            }
        }
        if (j + 1 < nsteps) load_gx(j + 1);
        __syncthreads();
        hb ^= 1;
        // ---- FC layers after the LSTM (rows tiles dealt over the RG waves)
        const int16_t* in = &R.h[hb][0][0];
        int cur = 0;
        for (int i = r.li + 1; i < img.nl; ++i) {
            const NnLayer& Ly = img.L[i];
            const uint8_t* A = W + (Ly.a_off - r.a_off);
            int16_t* out = &R.act[cur][0][0];
            v4i fh[2], fl[2];
            load_b<2>(in, R_STRIDE, Ly.nkt, lane, fh, fl);
            for (int rt = g; rt < Ly.nrt; rt += RG) {
                v4i ah = {0, 0, 0, 0}, al = {0, 0, 0, 0};
#pragma unroll
                for (int kt = 0; kt < 2; ++kt)
                    if (kt < Ly.nkt) {
                        const v4i w = *reinterpret_cast<const v4i*>(A + (size_t)(rt * Ly.nkt + kt) * 1024 + 16 * lane);
                        ah = mfma8(w, fh[kt], ah);
                        al = mfma8(w, fl[kt], al);
                    }
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int row = 16 * rt + 4 * q + e;
                    if (row >= Ly.rows) continue;
                    const int32_t sum = (ah[e] << 8) + al[e] + img.wsum[Ly.ep_off + row];
                    const int32_t v = affine_out(sum, img.bias[Ly.ep_off + row], Ly, img.acc32);
                    if (Ly.act == ACT_LINEAR)
                        reinterpret_cast<int32_t*>(out + sc * R_STRIDE)[row] = v;
                    else
                        out[sc * R_STRIDE + row] = act16(Ly.act, v, tt);
                }
            }
            __syncthreads();
            in = out;
            cur ^= 1;
        }
        // ---- outputs and post-processing (nn_speech.c:92-124), wave 0 of the tile
        if (g == 0) {
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
        __syncthreads();
    }
    // ---- state out
    for (int idx = g * 64 + lane; idx < 16 * N; idx += 64 * RG) {
        const int st = idx / N, u = idx - st * N;
        if (i0 + st < nrow) {
            const int gs = sid(i0 + st);
            r.h[(size_t)gs * NN_MAX_W + u] = R.h[hb][st][u];
            r.c[(size_t)gs * NN_MAX_W + u] = R.c[st][u];
        }
    }
    if (g == 0 && lane < 16 && valid && b < e) {
        ps.slides = (int16_t)(ps.slides ^ ((e - b) & 1));
        reinterpret_cast<PostState*>(r.post)[s] = ps;
    }
}

extern "C" {

size_t nnspk_fast_lds_bytes(int which, int a_bytes, int units) {
    // which 0: proj (units = waves); 1: recur (units = tiles per workgroup)
    if (which == 0) return (size_t)a_bytes + 768 + (size_t)units * sizeof(ProjWave);
    return (size_t)a_bytes + 768 + (size_t)units * sizeof(RecTile);
}

int nnspk_launch_proj(const NnImage* img, const FastRun* r, int blocks, void* stream) {
    const size_t lds = nnspk_fast_lds_bytes(0, r->a_lds_bytes, 4);
    hipLaunchKernelGGL(proj_kernel, dim3(blocks), dim3(256), lds, (hipStream_t)stream, *img, *r);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

int nnspk_launch_recur(const NnImage* img, const FastRun* r, int tpw, void* stream) {
    const size_t lds = nnspk_fast_lds_bytes(1, r->a_lds_bytes, tpw);
    const int nrow = r->list ? r->n_list : r->S;
    if (nrow <= 0) return 0;
    const int tiles = (nrow + 15) / 16;
    const int blocks = (tiles + tpw - 1) / tpw;
    const int rpw = (img->L[r->li].nrt + RG - 1) / RG;
    const dim3 grid(blocks), blk(64 * RG * tpw);
    if (rpw <= 2)
        hipLaunchKernelGGL(recur_kernel<2>, grid, blk, lds, (hipStream_t)stream, *img, *r);
    else if (rpw <= 4)
        hipLaunchKernelGGL(recur_kernel<4>, grid, blk, lds, (hipStream_t)stream, *img, *r);
    else if (rpw <= 5)
        hipLaunchKernelGGL(recur_kernel<5>, grid, blk, lds, (hipStream_t)stream, *img, *r);
    else
        hipLaunchKernelGGL(recur_kernel<8>, grid, blk, lds, (hipStream_t)stream, *img, *r);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : (int)e;
}

int nnspk_set_lds_limit(void) {
    // allow up to 160 KiB of dynamic LDS for the split kernels
    hipError_t e = hipFuncSetAttribute((const void*)proj_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return (int)e;
    const void* ks[4] = {(const void*)recur_kernel<2>, (const void*)recur_kernel<4>,
                         (const void*)recur_kernel<5>, (const void*)recur_kernel<8>};
    for (int i = 0; i < 4; ++i) {
        e = hipFuncSetAttribute(ks[i], hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return (int)e;
    }
    return 0;
}

}  // extern "C"
