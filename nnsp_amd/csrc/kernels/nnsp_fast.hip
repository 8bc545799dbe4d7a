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
// A-fragments, with one folded epilogue constant per output row.
//
// Both kernels are compiled per net shape (tile counts known at compile time:
// loops unroll, LDS loads batch, no per-row branches) for the three reference
// shapes, plus a generic instantiation that reads the shape at run time.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <type_traits>

#include "nnsp_dev.h"
#include "nnsp_kabi.h"
#include "nnsp_casc.h"
#include "nnsp_nn.h"

using namespace nnsp;

// development probes (NNSP_RECUR_CLOCKS: s_memtime per phase), compiled in
// only with -DNNSP_PROBES=1 (make PROBES=1; profiles/recur_clocks.py).  Their
// pointer and bound checks cost the loops SGPRs: built in, the recurrence
// kernels spilled 40-60 SGPRs to VGPR lanes (10 without them) and read them
// back with v_readlane in the step loops
#ifndef NNSP_PROBES
#define NNSP_PROBES 0
#endif
#define TT_BYTES ACT_BYTES   // LDS copy of nnsp_tbl_act (act_q15) at LDS offset 0, before the staged A fragments
                               // (a compile-time address: the lookups need no base add)
#define P_ASTRIDE 264   // int16 per row of a proj activation buffer
#define P_UNION 1920    // context frames of a tile: G streams x (32/G + 4) frames x 40 features (int16)
#define R_STRIDE 136    // int16 per row of recur h / activation buffers
#define R_CW 128        // int32 per row of the c buffer (before cstride)

// int32 row stride of a [16 streams][units] cell-state buffer: twice an odd
// number, so that the 32 lanes of a ds_read_b32 / ds_write_b32 lane group
// (q = 0, 1 or 2, 3 and the 16 streams sc) reaching unit 4 rt + q of row sc
// hit bank (stride * sc + 4 rt + q) mod 32 -- all 32 distinct (MI355X_MICROARCH
// LDS table: b32 accesses bank by dword mod 32 in two groups of 32 lanes).  A
// stride of 64 (KWS) put the 16 streams of a unit on one bank: 16-way
// conflicts on every cell-state load and store (round 4 PMC: 5.0 conflict
// cycles per LDS instruction in KWS's recurrence)
__host__ __device__ constexpr int cstride(int units) {
    return ((units + 1) / 2) % 2 ? (units + 1) / 2 * 2 : (units + 1) / 2 * 2 + 2;
}

// ---------------------------------------------------------------------------
// Net shapes.  NRT == 0: generic (read from the NnLayer table at run time).
//   NKR   K tiles (64) of the LSTM input and recurrent halves (N <= 128)
//   NRT   LSTM row tiles (4N rows / 16)
//   R0    row tiles of the FC layer before the LSTM (K = 240: 4 K tiles)
//   R1,R2 row tiles of the two relu6 FC layers after the LSTM (K = N)
//   R3    row tiles of the linear output layer; NW = N, NOUT = its width
// ---------------------------------------------------------------------------
template <int NKR_, int NRT_, int R0_, int R1_, int R2_, int R3_, int NW_, int NOUT_>
struct Shape {
    static constexpr bool generic = NRT_ == 0;
    static constexpr int NKR = NKR_, NRT = NRT_, R0 = R0_, R1 = R1_, R2 = R2_, R3 = R3_, NW = NW_, NOUT = NOUT_;
    static constexpr int RPW = (NRT_ + 3) / 4;
    static constexpr int XS = (NW_ + 15) / 16 * 16;   // int16 per x row (proj -> recur, compiled shapes)
};
using ShapeGen = Shape<0, 0, 0, 0, 0, 0, 0, 0>;
using ShapeVad = Shape<1, 7, 2, 2, 2, 1, 28, 2>;      // def_nn1_vad.c
using ShapeKws = Shape<1, 16, 4, 4, 4, 1, 64, 2>;     // def_nn2_kws_galaxy.c
using ShapeS2i = Shape<2, 18, 5, 5, 5, 3, 72, 41>;    // def_nn0_s2i.c

// ---------------------------------------------------------------------------
// Folded epilogue constants.  affine_Krows_8x16 (affine.c:74-248) computes
// s = sum_k W x + (b << (qbit_s - qb)), then shift_64b/32b; the MFMA tiles
// deliver acc = sum_k W (x - 128) exactly, so per row
//   cst = 128 * sum_k W + bias term        (int64; int32 wrap for acc32)
// and the layer output is shift(acc + cst).  For the LSTM input half the proj
// kernel needs the exact sum only (cst = 128 * sum_k Wx, no bias); the recur
// kernel folds the bias into the recurrent half (cst = 128 * sum_k Wh + bias).
// ---------------------------------------------------------------------------
struct EpRow {
    int64_t cst;
};

// recur: the LSTM rows' constant covers the recurrent half (and, xsum, the
// input half too: the compiled shapes' recur computes Wx.x itself)
__device__ __forceinline__ void stage_ep(EpRow* ep, const NnImage& img, int lo, int n, bool recur, bool xsum = false) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int row = lo + i;
        int li = 0;
        while (li + 1 < img.nl && img.L[li + 1].ep_off <= row) ++li;
        const NnLayer& Ly = img.L[li];
        const bool lstm = Ly.type == NN_LSTM;
        int64_t bt = 0;
        if (Ly.has_bias && (recur || !lstm)) {
            const int16_t b = img.bias[row];
            if (img.acc32)
                bt = Ly.bias_sh >= 0 ? wshl(b, Ly.bias_sh) : ((int32_t)b >> -Ly.bias_sh);
            else
                bt = Ly.bias_sh >= 0 ? (int64_t)((uint64_t)(int64_t)b << Ly.bias_sh) : ((int64_t)b >> -Ly.bias_sh);
        }
        const int32_t w = lstm && recur ? (xsum ? wadd(img.wsum_r[row], img.wsum[row]) : img.wsum_r[row])
                                        : img.wsum[row];
        ep[i].cst = img.acc32 ? (int64_t)wadd(w, (int32_t)bt) : (int64_t)w + bt;
    }
}

__host__ __device__ inline size_t ep_bytes(int n) { return ((size_t)n * sizeof(EpRow) + 15) & ~(size_t)15; }

// epilogue constant as the kernel consumes it: the int32 accumulator kernels
// wrap-add only its low word (ep_out<true>), so they load 4 bytes of it
template <bool ACC32>
using CstT = typename std::conditional<ACC32, int32_t, int64_t>::type;
template <bool ACC32>
__device__ __forceinline__ CstT<ACC32> ep_cst(const EpRow& e) {
    if constexpr (ACC32)
        return reinterpret_cast<const int32_t*>(&e.cst)[0];
    else
        return e.cst;
}

// shift_64b + clamp (acc64) or shift_32b (acc32) of acc + cst.  rsh/lsh = the
// layer's output shift split by sign (lsh > 0 never happens for the reference nets).
template <bool ACC32>
__device__ __forceinline__ int32_t ep_out(int32_t acc, int64_t cst, int rsh, int lsh) {
    if (ACC32) {
        const int32_t v = wadd(acc, (int32_t)cst);
        return __builtin_expect(lsh > 0, 0) ? shift32(v, lsh) : (v >> rsh);
    }
    const int64_t v = (int64_t)acc + cst;
    return sat32(__builtin_expect(lsh > 0, 0) ? shift64(v, lsh) : (v >> rsh));
}

__device__ __forceinline__ void stage_weights(uint8_t* dst, const uint8_t* src, int bytes) {
    const int4* s = reinterpret_cast<const int4*>(src);
    int4* d = reinterpret_cast<int4*>(dst);
    for (int i = threadIdx.x; i < bytes / 16; i += blockDim.x) d[i] = s[i];
}

// Row tiles per load group of a compiled-shape FC layer: all of a layer's
// tiles (up to FC_GROUP_MAX) in one group, so that its LDS loads and MFMA
// chains overlap once instead of once per group of 3.
#ifndef FC_GROUP_MAX
#define FC_GROUP_MAX 3
#endif
// One FC layer on a 16-row tile: B from an LDS buffer (row stride in_stride),
// A fragments from LDS, output to an LDS buffer (row stride out_stride).
// NRT/NKT/ROWS > 0 and ACT >= 0 are compile-time; otherwise taken from Ly.
// PAD (compiled shapes): also compute and store the padding rows of the last
// row tile (rows .. 16 NRT - 1; their epilogue constants are zero), so that no
// output store sits behind a lane-dependent branch.  Only for outputs whose
// row stride holds 16 NRT values and whose padding only ever meets zero A
// columns of the next layer (recur's stage buffers).
template <bool ACC32, int NRT, int NKT, int ACT, int ROWS, int MAXKT, bool PAD = false>
__device__ __forceinline__ void fc_layer(const NnLayer& Ly, const uint8_t* A, const EpRow* ep, const int16_t* in,
                                         int in_stride, int16_t* out, int out_stride, const uint8_t* tt, int lane) {
    const int nrt = NRT > 0 ? NRT : Ly.nrt;
    const int nkt = NKT > 0 ? NKT : Ly.nkt;
    const int act = ACT >= 0 ? ACT : Ly.act;
    const int rows = ROWS > 0 ? ROWS : Ly.rows;
    const int rsh = Ly.out_sh < 0 ? -Ly.out_sh : 0, lsh = Ly.out_sh > 0 ? Ly.out_sh : 0;
    v4i bh[MAXKT], bl[MAXKT];
    load_b<MAXKT>(in, in_stride, nkt, lane, bh, bl);
    const int sc = lane & 15, q = lane >> 4;
    auto tile = [&](int rt) {
        v4i ah = {0, 0, 0, 0}, al = {0, 0, 0, 0};
#pragma unroll
        for (int kt = 0; kt < MAXKT; ++kt)
            if (kt < nkt) {
                const v4i w = *reinterpret_cast<const v4i*>(A + (size_t)(rt * nkt + kt) * 1024 + 16 * lane);
                ah = mfma8(w, bh[kt], ah);
                al = mfma8(w, bl[kt], al);
            }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = 16 * rt + 4 * q + i;
            if (row < rows) {
                const int32_t v = ep_out<ACC32>((ah[i] << 8) + al[i], ep[row].cst, rsh, lsh);
                if (act == ACT_LINEAR)
                    reinterpret_cast<int32_t*>(out + sc * out_stride)[row] = v;
                else
                    out[sc * out_stride + row] = act16s(act, v, tt);
            }
        }
    };
    if constexpr (NRT > 0 && NKT > 0) {
        // compiled shape: the LDS loads of a group of row tiles (A fragments,
        // epilogue constants) are issued before the group's first output
        // store -- the compiler cannot move loads across stores into the same
        // LDS, so a per-tile load/compute/store order would expose the full
        // latency per tile; groups of <= 3 tiles bound the registers
        constexpr int CH = NRT <= FC_GROUP_MAX ? NRT : 3;
#pragma unroll
        for (int r0 = 0; r0 < NRT; r0 += CH) {
            v4i w[CH][NKT];
            CstT<ACC32> cst[CH][4];
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                const int rt = r0 + c;
                if (rt < NRT) {
#pragma unroll
                    for (int kt = 0; kt < NKT; ++kt)
                        w[c][kt] = *reinterpret_cast<const v4i*>(A + (size_t)(rt * NKT + kt) * 1024 + 16 * lane);
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int row = 16 * rt + 4 * q + i;
                        cst[c][i] = (PAD || row < rows) ? ep_cst<ACC32>(ep[row]) : 0;
                    }
                }
            }
            // ACC32: each row's epilogue constant starts its low-plane
            // accumulator (mod 2^32 the same sum, as the recurrence's gates), so
            // the epilogue adds nothing
            v4i ah[CH], al[CH];
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                ah[c] = v4i{0, 0, 0, 0};
                al[c] = ACC32 ? v4i{(int32_t)cst[c][0], (int32_t)cst[c][1], (int32_t)cst[c][2], (int32_t)cst[c][3]}
                              : v4i{0, 0, 0, 0};
                if (r0 + c < NRT)
#pragma unroll
                    for (int kt = 0; kt < NKT; ++kt) {
                        ah[c] = mfma8(w[c][kt], bh[kt], ah[c]);
                        al[c] = mfma8(w[c][kt], bl[kt], al[c]);
                    }
            }
            // int32 accumulators without a left shift (every int32 kernel of
            // the reference nets): shift_32b is a plain arithmetic shift, so
            // no per-value select between the two shift forms
            const int rsh3 = min(rsh + 3, 31);   // (v >> rsh) >> 3 == v >> min(rsh + 3, 31)
            auto epilogue = [&](auto nolsh) {
#pragma unroll
                for (int c = 0; c < CH; ++c)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int row = 16 * (r0 + c) + 4 * q + i;
                        if (r0 + c < NRT && (PAD || row < rows)) {
                            const int32_t acc = (ah[c][i] << 8) + al[c][i];   // (+ cst: ACC32)
                            int32_t v;
                            if constexpr (decltype(nolsh)::value) {
                                if (act == ACT_RELU6) {   // relu6_q12's >> 3 folded into the layer shift
                                    const int32_t u = acc >> rsh3;
                                    out[sc * out_stride + row] = (int16_t)min(max(u, 0), 24576);
                                    continue;
                                }
                                v = acc >> rsh;
                            } else {
                                v = ep_out<ACC32>(acc, ACC32 ? 0 : cst[c][i], rsh, lsh);
                            }
                            if (act == ACT_LINEAR)
                                reinterpret_cast<int32_t*>(out + sc * out_stride)[row] = v;
                            else
                                out[sc * out_stride + row] = act16s(act, v, tt);
                        }
                    }
            };
            if (ACC32 && lsh == 0)
                epilogue(std::true_type{});
            else
                epilogue(std::false_type{});
        }
    } else if constexpr (NRT > 0) {
#pragma unroll
        for (int rt = 0; rt < NRT; ++rt) tile(rt);
    } else {
        for (int rt = 0; rt < nrt; ++rt) tile(rt);
    }
}


// per-frame results of stream s at frame f (NNSPClass_exec's return value and
// NNSPClass.outputs after the frame): per-net buffers for the controller and,
// in a cascade, the caller's outputs
__device__ __forceinline__ void put_out(const FastRun& r, int s, int T, int f, int16_t trig, int16_t o0, int16_t o1,
                                        int16_t o2) {
    const size_t i = (size_t)s * T + f;
    if (r.trig) r.trig[i] = trig;
    if (r.out3) {
        r.out3[i * 3] = o0;
        r.out3[i * 3 + 1] = o1;
        r.out3[i * 3 + 2] = o2;
    }
    if (r.detected) r.detected[i] = trig;
    if (r.net_ran) r.net_ran[i] = (int8_t)r.net_id;
    if (r.outputs3) {
        r.outputs3[i * 3] = o0;
        r.outputs3[i * 3 + 1] = o1;
        r.outputs3[i * 3 + 2] = o2;
    }
}
__device__ __forceinline__ void put_frame(const FastRun& r, int s, int T, int f, const PostState& ps) {
    put_out(r, s, T, f, ps.trigger, ps.outputs[0], ps.outputs[1], ps.outputs[2]);
}
// ---------------------------------------------------------------------------
// proj_kernel
// ---------------------------------------------------------------------------
// Per-wave LDS of proj.  The compiled shapes keep one activation buffer as
// wide as the LSTM input's K tiles (+8: rows 16 B apart modulo 256 B); the
// generic shape ping-pongs two full-width buffers across its prefix layers.
//
// Compiled shapes: two union buffers, the next tile's features loading into
// one (LDS-DMA) while the current tile computes from the other; a tile's
// activations overwrite its own union once the FC layer has read it (the
// B operand is loaded before the first output store), so the act rows need
// no buffer of their own.
//
// Per G (streams per tile) the union holds G x (32/G + 4) context frames; the
// descriptor pipeline's slots (pd) take what the tile loop loads ahead by
// LDS-DMA: per tile parity, lanes 0..G-1, the list entry, segment start,
// post-state dword (slides) and fresh[] dword.
template <class SH, int G = 1>
struct alignas(16) ProjWave {
    static constexpr int AS = SH::generic ? P_ASTRIDE : 64 * SH::NKR + 8;
    static constexpr int NA = SH::generic ? 2 : 1;
    static constexpr int PU = SH::generic ? P_UNION : G * (32 / G + 4) * 40;      // union int16 of a G tile
    static constexpr int UNI = (PU + 32) > 16 * AS ? (PU + 32) : 16 * AS;   // int16 per union buffer
    int16_t uni[SH::generic ? 1 : 2][SH::generic ? P_UNION + 32 : UNI];
    int16_t act[SH::generic ? NA : 0][16][AS];
    int32_t pd[SH::generic ? 0 : 2][4][4];   // [parity][list, seg_begin, post dword, fresh dword][lane < G]
};

// LDS-DMA (global_load_lds) of BYTES per lane at lds + lane * BYTES, issued
// from inline asm: the compiler then inserts no wait of its own for it.  With
// the builtin it put a vmcnt(0) before the first LDS access after the DMA --
// it cannot tell the buffer being filled from the one being read -- so the
// next tile's loads were waited for before this tile's compute.  The caller
// waits (s_waitcnt vmcnt) before reading what it DMA'd.  M0 is saved and
// restored around it.
template <int BYTES>
__device__ __forceinline__ void lds_dma(const void* g, void* lds) {
    static_assert(BYTES == 4 || BYTES == 16, "lds_dma: dword or dwordx4");
    const unsigned l =
        __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)lds);
    unsigned saved;
    if constexpr (BYTES == 16)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(saved) : "v"(g), "s"(l) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(saved) : "v"(g), "s"(l) : "memory");
}

// 16 bytes through a global (not flat) load: flat loads also count in lgkmcnt
// and complete out of order, so the compiler waits for them (and everything
// else) at once
__device__ __forceinline__ int4 gload16(uintptr_t a) {
    const v4i v = *reinterpret_cast<const __attribute__((address_space(1))) v4i*>(a);
    return make_int4(v.x, v.y, v.z, v.w);
}

// 16 zero bytes: the source of union elements outside a segment (proj_kernel)
__device__ __attribute__((aligned(16))) int4 nnsp_proj_zero16;
// where proj's x-row stores of rows without an NN step go (>= XS + 8 bytes)
__device__ __attribute__((aligned(16))) uint2 nnsp_proj_sink[32];
__device__ int32_t nnsp_proj_neg1 = -1;   // the list entry of a tile slot past the list

// GT: streams per 16-row tile (compiled shapes: 1, 2 or 4, FastRun.gpt; one
// instantiation each, so a G = 1 tile's descriptors are wave-uniform scalars)
template <class SH, bool ACC32, int GT>
__global__ __launch_bounds__(512, 4) void proj_kernel(NnImage img, FastRun r) {   // <= 128 VGPRs: 4 waves per SIMD
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* W = smem + TT_BYTES;                                           // staged A fragments
    const uint8_t* tt = smem;   // act_q15 tables
    EpRow* ep = reinterpret_cast<EpRow*>(smem + r.a_lds_bytes + TT_BYTES);
    constexpr bool GEN = SH::generic;
    using PW = ProjWave<SH, GEN ? 1 : GT>;
    PW* pw = reinterpret_cast<PW*>(smem + r.a_lds_bytes + TT_BYTES + ep_bytes(r.ep_n));
    // wave-uniform tile arithmetic (32-bit, scalar): with the wave index in a
    // VGPR every tile paid three 64-bit divisions on the VALU (~250 VALU per tile)
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nwv = blockDim.x >> 6;
    PW& P = pw[wv];
    const int sc = lane & 15, q = lane >> 4;
    const NnLayer& LL = img.L[r.li];
    const int nrt = GEN ? LL.nrt : SH::NRT;
    const int nkt = GEN ? LL.nkt : SH::NKR;
    const int rows = 16 * nrt;   // LSTM rows are padded to whole tiles (4 units per group)
    const int wsteps = r.seg_len > 0 ? min(r.nstep_max, (r.seg_len + 1) / 2) : r.nstep_max;
    // a 16-row MFMA tile is G streams x SPT consecutive NN steps: G = 1 tiles
    // a stream's steps 16 at a time; short segments (cascade rounds, host:
    // SPT >= the segment's steps) pack G = 2 or 4 streams into one tile
    constexpr int G = GEN ? 1 : GT;
    constexpr int SPT = 16 / G;
    constexpr int FR = 2 * SPT + 4;                   // context frames of one stream's rows
    const int ntps = (wsteps + SPT - 1) / SPT;        // tiles per group of G streams
    const int nrow = r.n_list_dev ? *r.n_list_dev : (r.list ? r.n_list : r.S);
    if (r.n_list_rec && blockIdx.x == 0 && threadIdx.x == 0) *r.n_list_rec = nrow;
    const int ngrp = (nrow + G - 1) / G;
    const int ntiles = ngrp * ntps;   // < 2^31: S * T < 2^31 (host)
    // device-sized lists (cascade rounds): workgroups with no tile exit
    // before staging anything
    if ((int)blockIdx.x * nwv >= ntiles) return;
    // development probe (NNSP_RECUR_CLOCKS): per wave, wall clock (100 MHz) at
    // the start, after staging, at the end, and the tiles it ran
    const unsigned pwid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    long long* pwc = (NNSP_PROBES && r.dbg_clk && lane == 0 && pwid < 8192u) ? r.dbg_clk + 2048 + 4 * 32768 + 4 * pwid : nullptr;
    if (pwc) pwc[0] = (long long)__builtin_amdgcn_s_memrealtime();
    stage_weights(W, img.A + r.a_off, r.a_lds_bytes);
    stage_ep(ep, img, r.ep_lo, r.ep_n, false);
    for (int i = threadIdx.x; i < TT_BYTES / 16; i += blockDim.x)
        reinterpret_cast<int4*>(smem)[i] = reinterpret_cast<const int4*>(nnsp_tbl_act)[i];
    __syncthreads();
    if (pwc) pwc[1] = (long long)__builtin_amdgcn_s_memrealtime();
    int ntile_run = 0;
    // stream k of a tile: list entry, segment start b, length L, NN phase,
    // fresh[] (cascade: frames since the net's reset, 0..2; 2 otherwise) --
    // loaded with the descriptors, ahead: read in the union loads, it made
    // every union chunk wait (vmcnt(0)) for it, the loads before it and the
    // last tile's x stores
    struct Seg { int s, b, L, ph; bool ok; int fr; };
    // development probe (NNSP_RECUR_CLOCKS): s_memtime per phase of wave 0's first tiles
    long long* clk = (NNSP_PROBES && r.dbg_clk && blockIdx.x == 0 && wv == 0 && lane == 0) ? r.dbg_clk + 12 : nullptr;
    int it = 0;
#define PCLK(k) \
    if (clk && it < 64) clk[it * 16 + (k)] = (long long)__builtin_amdgcn_s_memtime()
    // The tiles run as a software pipeline over their descriptors.  A tile's
    // inputs are a chain of dependent loads (list entry -> segment start and
    // phase -> the context features): one tile at a time exposed three HBM
    // latencies per tile (~4.5 us per tile and wave).  The list entries are
    // loaded two tiles ahead and the segment descriptors one tile ahead, so a
    // tile waits only for its features.  (Prefetching the features as well
    // took 16 more VGPRs per lane held across the FC layer: past 128, spills.)
    const int tstride = (int)gridDim.x * nwv;
    auto grp_of = [&](int t) { return ntps == 1 ? t : (ntps == 4 ? t >> 2 : (ntps == 2 ? t >> 1 : t / ntps)); };
    auto j0_of = [&](int t) { return SPT * (t - grp_of(t) * ntps); };
    // lanes 0..G-1: the tile's stream k = lane (the others read by shuffle); -1: none
    auto list_at = [&](int t) {
        if (t >= ntiles) return -1;
        const int i = G == 1 ? grp_of(t) : grp_of(t) * G + (lane < G ? lane : 0);
        return i < nrow ? (r.list ? r.list[i] : (int)i) : -1;
    };
    auto seg_from = [&](int st) {
        Seg g;
        g.ok = st >= 0;
        g.s = g.ok ? st : 0;
        g.b = g.ok && r.seg_begin ? r.seg_begin[g.s] : 0;
        g.L = g.ok ? (r.seg_len > 0 ? min(r.T, g.b + r.seg_len) : r.T) - g.b : 0;
        g.ph = g.ok ? 1 - reinterpret_cast<const NnPost*>(r.post)[g.s].slides : 0;
        g.fr = g.ok && r.fs.nring ? min((int)r.fs.fresh[g.s], 2) : 2;
        return g;
    };
    int tile = (int)blockIdx.x * nwv + wv;
    if constexpr (!GEN) {
        // ---- compiled shapes: the next tile's features (LDS-DMA into the
        //      other union buffer) and descriptors load while this tile
        //      computes; one vmcnt(0) per tile then waits only for what was
        //      issued a whole tile earlier (and the x stores of the last one)
        constexpr int XC = SH::XS / 8;   // 8-element chunks of an x row
        // the union of tile t (descriptor m) into buffer bf; false: no row of
        // the tile has a frame (wave-uniform), nothing issued
        auto union_issue = [&](const Seg& m, int t, int bf) -> bool {
            const int j0 = j0_of(t);
            if (!__any(lane < G && m.ok && 2 * j0 + m.ph < m.L)) return false;
            const Seg g1 = {__builtin_amdgcn_readfirstlane(m.s), __builtin_amdgcn_readfirstlane(m.b),
                            __builtin_amdgcn_readfirstlane(m.L), __builtin_amdgcn_readfirstlane(m.ph),
                            __builtin_amdgcn_readfirstlane((int)m.ok) != 0, __builtin_amdgcn_readfirstlane(m.fr)};
            constexpr int NU = G * FR * 5;   // 16-byte chunks (8 features) of the union
            if constexpr (G == 1) {
                // one stream whose window V[t0 .. t0 + FR) lies past prev5 and
                // past the segment's (possibly cold) first two frames: its
                // features are consecutive frames of the ring (or of feats),
                // chunk c = 5d + part at frame t0 + d.  Frames past the
                // segment feed only rows that are not stored: they re-read the
                // segment's last frame (in bounds) instead of a zero row.
                const int t0 = 2 * j0 + g1.ph;
                if (t0 >= 7) {
                    const int dmax = g1.L + 4 - t0;             // V index L + 4: the segment's last frame
                    const int f0 = g1.b + t0 - 5;               // chunk frame of V[t0]
                    const bool ring = r.fs.nring != nullptr;
                    const unsigned rg = ring ? (unsigned)r.fs.ring : 0u;
                    unsigned slot0 = 0;
                    if (ring) {   // (abs0 + f0 - lookback) mod ring, as feat8_ptr
                        slot0 = (unsigned)(r.fs.abs0 + f0 - r.fs.lookback) + rg;
                        slot0 = slot0 >= rg ? slot0 - rg : slot0;
                        slot0 = slot0 >= rg ? slot0 - rg : slot0;
                    }
                    const char* base = ring ? reinterpret_cast<const char*>(r.fs.nring) + (size_t)g1.s * rg * 80
                                            : reinterpret_cast<const char*>(r.feats) + ((size_t)g1.s * r.T + f0) * 80;
#pragma unroll
                    for (int mm = 0; mm < (NU + 63) / 64; ++mm) {
                        const int c = lane + 64 * mm;
                        if (mm < NU / 64 || c < NU) {
                            const int d0 = (c * 52429) >> 18;   // c / 5 (c < 2^14)
                            const int part = c - 5 * d0;
                            const unsigned d = (unsigned)min(d0, dmax);
                            unsigned row = d;
                            if (ring) {
                                row = slot0 + d;
                                row = row >= rg ? row - rg : row;
                            }
                            const char* src = base + (row * 80u + 16u * (unsigned)part);
                            lds_dma<16>(src, &P.uni[bf][512 * mm]);
                        }
                    }
                    return true;
                }
            }
#pragma unroll
            for (int mm = 0; mm < (NU + 63) / 64; ++mm) {
                int c = lane + 64 * mm;
                asm volatile("" : "+v"(c));
                if (mm < NU / 64 || c < NU) {
                    const int k = c / (FR * 5), rem = c - k * (FR * 5), fr = rem / 5, part = rem - 5 * fr;
                    Seg g = g1;
                    if (G > 1) {
                        g.s = __shfl(m.s, k);
                        g.b = __shfl(m.b, k);
                        g.L = __shfl(m.L, k);
                        g.ph = __shfl(m.ph, k);
                        g.ok = __shfl((int)m.ok, k) != 0;
                        g.fr = __shfl(m.fr, k);
                    }
                    const int idx = 2 * j0 + g.ph + fr;
                    const int16_t* src = reinterpret_cast<const int16_t*>(&nnsp_proj_zero16);
                    if (g.ok) {
                        if (idx < 5)
                            src = r.prev5 + ((size_t)g.s * 5 + idx) * 40 + 8 * part;
                        else if (idx - 5 < g.L)
                            src = feat8_ptr<true>(r.fs, r.feats, g.s, r.T, g.b, g.b + idx - 5, part, g.fr);
                    }
                    lds_dma<16>(src, &P.uni[bf][512 * mm]);
                }
            }
            return true;
        };
        // The descriptor pipeline, in LDS: every load of it lands by LDS-DMA
        // (global_load_lds, tracked like the union's loads by the top-of-tile
        // wait; the compiler tracks none of it), so no register waits on an
        // in-flight load.  At the top of tile t: the slots of tile t+1 (DMA'd a
        // tile earlier) give its descriptor, whose union then loads; the list
        // entries of tile t+2 (DMA'd a tile earlier) address the DMA of its
        // segment start, post-state and fresh[] dwords; the list entries of
        // tile t+3 are DMA'd.  (Until round 4 the descriptors went through
        // registers: each tile waited out one memory latency for them, and the
        // loop-carried copies waited for the last tile's stores.)
        // Slot parity: tile it + k -> pd[(it + k) & 1].
        const int* dz = reinterpret_cast<const int*>(&nnsp_proj_zero16);
        auto dma4 = [&](const void* src, int32_t* dst) { lds_dma<4>(src, dst); };   // lanes < G: dst[lane]
        auto list_dma = [&](int t, int slot) {   // list entry of tile t (-1: none) -> pd[slot][0]
            const int i = grp_of(t) * G + (lane < G ? lane : 0);
            const bool ok = t < ntiles && i < nrow;
            if (r.list) {
                if (lane < G) dma4(ok ? (const void*)(r.list + i) : (const void*)&nnsp_proj_neg1, &P.pd[slot][0][0]);
            } else if (lane < G) {
                P.pd[slot][0][lane] = ok ? i : -1;
            }
        };
        auto desc_dma = [&](int st, int slot) {   // st: lane's stream (lanes < G) -> pd[slot][1..3]
            if (lane < G) {
                const int q = st >= 0 ? st : 0;
                dma4(st >= 0 && r.seg_begin ? (const void*)(r.seg_begin + q) : (const void*)dz, &P.pd[slot][1][0]);
                dma4(st >= 0 ? (const void*)(reinterpret_cast<const NnPost*>(r.post) + q) : (const void*)dz,
                     &P.pd[slot][2][0]);
                dma4(st >= 0 && r.fs.nring ? (const void*)(r.fs.fresh + (q & ~3)) : (const void*)dz, &P.pd[slot][3][0]);
            }
        };
        auto desc_of = [&](int slot) {   // the descriptor in pd[slot] (lanes < G; G = 1: uniform)
            const int k = lane < G ? lane : 0;
            Seg g;
            const int st = P.pd[slot][0][k];
            g.ok = st >= 0;
            g.s = g.ok ? st : 0;
            g.b = g.ok ? P.pd[slot][1][k] : 0;
            g.L = g.ok ? (r.seg_len > 0 ? min(r.T, g.b + r.seg_len) : r.T) - g.b : 0;
            g.ph = g.ok ? 1 - (int)(int16_t)(P.pd[slot][2][k] & 0xffff) : 0;
            const int fr = (int)(int8_t)((unsigned)P.pd[slot][3][k] >> (8 * (g.s & 3)));
            g.fr = g.ok && r.fs.nring ? min(max(fr, 0), 2) : 2;
            if (G == 1) {   // wave-uniform: scalars
                g.s = __builtin_amdgcn_readfirstlane(g.s);
                g.b = __builtin_amdgcn_readfirstlane(g.b);
                g.L = __builtin_amdgcn_readfirstlane(g.L);
                g.ph = __builtin_amdgcn_readfirstlane(g.ph);
                g.fr = __builtin_amdgcn_readfirstlane(g.fr);
                g.ok = __builtin_amdgcn_readfirstlane((int)g.ok) != 0;
            }
            return g;
        };
        // x rows go out as a fixed number of store instructions per tile (rows
        // past the segment or the buffer to a sink), so the top-of-tile wait
        // for the next union need not wait for the last tile's stores: they
        // are the NST youngest vector memory operations
        constexpr int NST = 2 * ((16 * XC + 63) / 64);
        // prologue: tile `tile` with plain loads, the slots of tile + tstride
        // (descriptor) and tile + 2 tstride (list entry) by DMA, waited for
        Seg mine = seg_from(list_at(tile));
        list_dma(tile + tstride, (it + 1) & 1);
        list_dma(tile + 2 * tstride, it & 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        wave_lds_sync();
        desc_dma(lane < G ? P.pd[(it + 1) & 1][0][lane] : -1, (it + 1) & 1);
        bool have = tile < ntiles && union_issue(mine, tile, 0);
        bool stored = false;   // the last tile issued its NST x stores after this tile's union loads
        // two tiles per trip, the buffer and slot parity CB a template constant:
        // with a run-time parity the compiler could not tell the union being
        // read from the one being DMA'd and waited (vmcnt(0)) for the next
        // tile's loads before reading this tile's
        auto tile_step = [&](const int CB) {
            PCLK(0);
            // this tile's union landed, and every descriptor DMA issued before it
            if (stored && !clk)
                asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NST) : "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            wave_lds_sync();
            const Seg nxt = desc_of(CB ^ 1);                               // tile + tstride
            const int s2 = lane < G ? P.pd[CB][0][lane] : -1;                      // tile + 2 tstride
            // the slot reads above complete before the DMAs below write the slots
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            desc_dma(s2, CB);                                                // its descriptor
            if (lane < G) P.pd[CB][0][lane] = s2;                            // (kept beside it)
            list_dma(tile + 3 * tstride, CB ^ 1);                          // tile + 3 tstride
            // the next tile's union into the other buffer (its previous
            // contents, the last tile's x rows, were read into registers
            // for their stores before the wait above)
            const bool have_n = tile + tstride < ntiles && union_issue(nxt, tile + tstride, CB ^ 1);
            // keep the loads here, ahead of the compute (the compiler would
            // otherwise sink them below it: they write the other buffer)
            asm volatile("" ::: "memory");
            stored = false;
            if (have) {

                ++ntile_run;
                PCLK(1);
                const int j0 = j0_of(tile);
                auto seg_k = [&](int k) {
                    Seg g;
                    g.s = __shfl(mine.s, k);
                    g.b = __shfl(mine.b, k);
                    g.L = __shfl(mine.L, k);
                    g.ph = __shfl(mine.ph, k);
                    g.ok = __shfl((int)mine.ok, k) != 0;
                    g.fr = 2;
                    return g;
                };
                // ---- the prefix FC layer, K = 240, tanh (row (k, j)'s context =
                //      uni[k*FR*40 + 80j .. +239]; the per-lane base makes in +
                //      sc * 80 that row); its output rows overwrite the union
                const int kr = sc / SPT, jr = sc - kr * SPT;
                int16_t* U = &P.uni[CB][0];
                const int16_t* in = U + kr * FR * 40 + 80 * jr - 80 * sc;
                const NnLayer& L0 = img.L[0];
                // PAD: the last row tile's padding rows (N .. 16 R0 - 1) are
                // computed and stored too, with no per-value branch; the x
                // store below writes those columns as zeros
                fc_layer<ACC32, SH::R0, 4, ACT_TANH, SH::NW, 4, true>(L0, W + (L0.a_off - r.a_off),
                                                                    ep + (L0.ep_off - r.ep_lo), in, 80, U, PW::AS,
                                                                    tt, lane);
                wave_lds_sync();
                PCLK(2);
                // ---- the LSTM's input x of every row to HBM, already in the
                //      MFMA B operand's split form (split_hilo): per row xs high
                //      bytes, then xs low bytes ^ 0x80; columns N..xs-1 (not
                //      written by the layer) are stored as zeros.  Every lane
                //      stores (a row without a step to the sink): NST stores
#pragma unroll
                for (int c0 = 0; c0 < 16 * XC; c0 += 64) {
                    const int c = c0 + lane;
                    if (c0 + 64 <= 16 * XC || c < 16 * XC) {
                        const int row = c / XC, part = c - row * XC;
                        const int kx = row / SPT, jx = row - kx * SPT;
                        const Seg g = G == 1 ? mine : seg_k(kx);
                        const int j = j0 + jx;
                        const bool ok = g.ok && j < r.nstep_max && 2 * j + g.ph < g.L;
                        int4 v = *reinterpret_cast<const int4*>(U + row * PW::AS + 8 * part);
                        if (8 * XC > SH::NW && part == XC - 1) {   // mask the columns past N
                            int32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                            for (int e = 0; e < 4; ++e) {
                                const int col = 8 * part + 2 * e;
                                w4[e] = col + 1 < SH::NW ? w4[e] : (col < SH::NW ? (w4[e] & 0xffff) : 0);
                            }
                            v = make_int4(w4[0], w4[1], w4[2], w4[3]);
                        }
                        uintptr_t da = ok ? reinterpret_cast<uintptr_t>(
                                                reinterpret_cast<uint8_t*>(r.xg + ((size_t)g.s * r.nstep_max + j) * SH::XS) +
                                                8 * part)
                                          : reinterpret_cast<uintptr_t>(&nnsp_proj_sink[0]);
                        asm volatile("" : "+v"(da));   // one address per lane: keep the two stores unconditional
                        // global (not flat) stores: a flat store also counts in lgkmcnt
                        typedef __attribute__((address_space(1))) uint64_t gu64;
                        gu64* dst = reinterpret_cast<gu64*>(da);
                        const uint32_t HS = 0x07050301u, LS = 0x06040200u;
                        auto u64 = [](uint32_t lo, uint32_t hi) { return (uint64_t)lo | ((uint64_t)hi << 32); };
                        dst[0] = u64(__builtin_amdgcn_perm((uint32_t)v.y, (uint32_t)v.x, HS),
                                     __builtin_amdgcn_perm((uint32_t)v.w, (uint32_t)v.z, HS));
                        dst[SH::XS / 8] = u64(__builtin_amdgcn_perm((uint32_t)v.y, (uint32_t)v.x, LS) ^ 0x80808080u,
                                              __builtin_amdgcn_perm((uint32_t)v.w, (uint32_t)v.z, LS) ^ 0x80808080u);
                    }
                }
                stored = true;
                PCLK(3);
            }
            mine = nxt;
            have = have_n;
        };
        for (; tile < ntiles; tile += tstride, ++it) tile_step(it & 1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
    Seg mine_n = seg_from(list_at(tile));
    int s_nn = list_at(tile + tstride);
    for (; tile < ntiles; tile += tstride, ++it) {
        PCLK(0);
        const Seg mine = mine_n;
        mine_n = seg_from(s_nn);                     // the next tile's descriptors
        s_nn = list_at(tile + 2 * tstride);          // the list entries of the one after
        const int j0 = j0_of(tile);
        auto seg_k = [&](int k) {
            Seg g;
            g.s = __shfl(mine.s, k);
            g.b = __shfl(mine.b, k);
            g.L = __shfl(mine.L, k);
            g.ph = __shfl(mine.ph, k);
            g.ok = __shfl((int)mine.ok, k) != 0;
            return g;
        };
        // wave-uniform: skip a tile none of whose rows has a frame
        if (!__any(lane < G && mine.ok && 2 * j0 + mine.ph < mine.L)) continue;
        ++ntile_run;
        // ---- union of the context windows: stream k's rows read
        //      V_k[t0 .. t0 + FR - 1], V = prev5 ++ features[b..b+L), t0 = 2*j0 + phase.
        //      Loaded straight into LDS (global_load_lds: element c = lane + 64 m
        //      lands at uni + 16 c, lane-linear), no VGPRs, all in flight at once;
        //      elements outside a segment read a zero row.
        const Seg g1 = {__builtin_amdgcn_readfirstlane(mine.s), __builtin_amdgcn_readfirstlane(mine.b),
                        __builtin_amdgcn_readfirstlane(mine.L), __builtin_amdgcn_readfirstlane(mine.ph),
                        __builtin_amdgcn_readfirstlane((int)mine.ok) != 0};
        auto union_g = [&](auto GC) {
            constexpr int GG = decltype(GC)::value, FRG = 2 * (16 / GG) + 4, NU = GG * FRG * 5;
#pragma unroll
            for (int m = 0; m < (NU + 63) / 64; ++m) {
                // opaque per tile: hoisted out of the tile loop, the per-lane
                // element indices of the three G variants pinned ~70 VGPRs
                int c = lane + 64 * m;
                asm volatile("" : "+v"(c));
                if (m < NU / 64 || c < NU) {
                    const int k = c / (FRG * 5), rem = c - k * (FRG * 5), fr = rem / 5, part = rem - 5 * fr;
                    const Seg g = GG == 1 ? g1 : seg_k(k);   // one stream per tile: scalar
                    const int idx = 2 * j0 + g.ph + fr;
                    const int16_t* src = reinterpret_cast<const int16_t*>(&nnsp_proj_zero16);
                    if (g.ok) {
                        if (idx < 5)
                            src = r.prev5 + ((size_t)g.s * 5 + idx) * 40 + 8 * part;
                        else if (idx - 5 < g.L)
                            src = feat8_ptr(r.fs, r.feats, g.s, r.T, g.b, g.b + idx - 5, part);
                    }
                    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                                     (__attribute__((address_space(3))) void*)&P.uni[0][512 * m], 16, 0, 0);
                }
            }
        };
        if (G == 1)
            union_g(std::integral_constant<int, 1>{});
        else if (G == 2)
            union_g(std::integral_constant<int, 2>{});
        else
            union_g(std::integral_constant<int, 4>{});
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the LDS-DMA writes landed
        wave_lds_sync();
        PCLK(1);
        // this lane's row sc: stream kr of the tile, its step j0 + jr
        const int kr = sc / SPT, jr = sc - kr * SPT;
        const Seg me = seg_k(kr);
        // ---- prefix FC layers (row (k, j)'s context = uni[k*FR*40 + 80j .. +239];
        //      the per-lane base makes in + sc * in_stride that row)
        const int16_t* in = &P.uni[0][0] + kr * FR * 40 + 80 * jr - 80 * sc;
        int in_stride = 80;
        {
            for (int i = 0; i < r.li; ++i) {
                const NnLayer& Ly = img.L[i];
                int16_t* out = &P.act[i & (PW::NA - 1)][0][0];
                fc_layer<ACC32, 0, 0, -1, 0, 4>(Ly, W + (Ly.a_off - r.a_off), ep + (Ly.ep_off - r.ep_lo), in,
                                                in_stride, out, PW::AS, tt, lane);
                wave_lds_sync();
                in = out;
                in_stride = PW::AS;
            }
            // ---- LSTM input half (generic shape): gx = sum_k Wx[row][k] x[k] (exact, before shift_64b)
            v4i bh[2], bl[2];
            load_b<2>(in, in_stride, nkt, lane, bh, bl);
            const uint8_t* A = W + (LL.a_off - r.a_off);
            const EpRow* epl = ep + (LL.ep_off - r.ep_lo) + 4 * q;
            const int j = j0 + jr;
            const bool act = me.ok && j < r.nstep_max && 2 * j + me.ph < me.L;
            int32_t* dst = r.gx + ((size_t)me.s * r.nstep_max + j) * rows + 4 * q;
            for (int rt = 0; rt < nrt; ++rt) {
                v4i ah = {0, 0, 0, 0}, al = {0, 0, 0, 0};
#pragma unroll
                for (int kt = 0; kt < 2; ++kt)
                    if (kt < nkt) {
                        const v4i w = *reinterpret_cast<const v4i*>(A + (size_t)(rt * nkt + kt) * 1024 + 16 * lane);
                        ah = mfma8(w, bh[kt], ah);
                        al = mfma8(w, bl[kt], al);
                    }
                const EpRow* er = epl + 16 * rt;
                int4 o;
                o.x = (ah[0] << 8) + al[0] + (int32_t)er[0].cst;
                o.y = (ah[1] << 8) + al[1] + (int32_t)er[1].cst;
                o.z = (ah[2] << 8) + al[2] + (int32_t)er[2].cst;
                o.w = (ah[3] << 8) + al[3] + (int32_t)er[3].cst;
                if (act) *reinterpret_cast<int4*>(dst + 16 * rt) = o;
            }
            wave_lds_sync();
            PCLK(3);
        }
    }
    }
#undef PCLK
    if (pwc) {
        pwc[2] = (long long)__builtin_amdgcn_s_memrealtime();
        pwc[3] = (long long)ntile_run | (nnsp_hw_where() << 32);
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

// Per-tile LDS of recur; compiled shapes size the rows to their K tiles and
// the cell state to N (the generic shape to the widest net).
template <class SH>
struct alignas(16) RecTile {
    static constexpr int RS = SH::generic ? R_STRIDE : 64 * SH::NKR + 8;
    static constexpr int CW = cstride(SH::generic ? R_CW : SH::NW);
    int16_t h[2][16][RS];     // LSTM h, ping-pong across steps
    int16_t act[2][16][RS];   // tail wave: FC activations, ping-pong across layers
    int32_t c[16][CW];
    int32_t phase[16];
    int32_t nst[16];    // NN steps of each stream's segment
    int32_t beg[16];    // segment start frame
    int32_t end[16];    // segment end frame (exclusive)
};

// logits of one stream held in registers (post-processing without LDS round trips)
template <int N>
struct RegLogits {
    int32_t v[N];
    __device__ __forceinline__ int32_t operator[](int i) const { return v[i]; }
};

// logits of one stream read from its LDS row on use
struct LdsLogits {
    const int32_t* p;
    __device__ __forceinline__ int32_t operator[](int i) const { return p[i]; }
};

template <class SH, int RPW, bool ACC32>   // RPW: LSTM row tiles per wave = ceil(nrt / RG)
__global__ __launch_bounds__(64 * RW * 2) void recur_kernel(NnImage img, FastRun r) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr bool GEN = SH::generic;
    // tile = 16 consecutive entries of the stream list (identity when list == NULL)
    const int nrow = r.n_list_dev ? *r.n_list_dev : (r.list ? r.n_list : r.S);
    if ((int)(blockIdx.x * (blockDim.x / (64 * RW))) * 16 >= nrow) return;   // whole workgroup past the list
    uint8_t* W = smem + TT_BYTES;
    const uint8_t* tt = smem;   // act_q15 tables
    EpRow* ep = reinterpret_cast<EpRow*>(smem + r.a_lds_bytes + TT_BYTES);
    using RT = RecTile<SH>;
    constexpr int R_STRIDE_ = RT::RS;
    RT* tiles = reinterpret_cast<RT*>(smem + r.a_lds_bytes + TT_BYTES + ep_bytes(r.ep_n));
    stage_weights(W, img.A + r.a_off, r.a_lds_bytes);
    stage_ep(ep, img, r.ep_lo, r.ep_n, true);
    for (int i = threadIdx.x; i < TT_BYTES / 16; i += blockDim.x)
        reinterpret_cast<int4*>(smem)[i] = reinterpret_cast<const int4*>(nnsp_tbl_act)[i];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int tpw = blockDim.x / (64 * RW);
    const int tl = wv / RW, g = wv - tl * RW;   // tile in workgroup, wave in tile
    const bool tail = g == RG;
    RT& R = tiles[tl];
    const int sc = lane & 15, q = lane >> 4;
    const int i0 = (blockIdx.x * tpw + tl) * 16;
    auto sid = [&](int i) { return r.list ? r.list[i] : i; };
    const bool valid = i0 + sc < nrow;
    const int s = valid ? sid(i0 + sc) : 0;
    const NnLayer& LL = img.L[r.li];
    const int N = GEN ? LL.N : SH::NW;
    const int nrt = GEN ? LL.nrt : SH::NRT;
    const int nkt_r = GEN ? LL.nkt_r : SH::NKR;
    const int rows = 16 * nrt;
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
    if (tail && lane < 16 && valid && phase == 1 && b < e) put_frame(r, s, T, b, ps);   // frame b: no NN, trigger carried
    const uint8_t* Ar = W;   // LSTM recurrent fragments lead the staged region
    const EpRow* epl = ep + (LL.ep_off - r.ep_lo) + 4 * q;
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
    long long* clk = (r.dbg_clk && blockIdx.x == 0 && tl == 0 && (g == 0 || tail)) ? r.dbg_clk + (tail ? 8 : 0)
                                                                                     : nullptr;
#define PROBE(k) \
    if (clk && j < 64) clk[j * 16 + (k)] = (long long)__builtin_amdgcn_s_memtime()
    int cur = 0;
    for (int j = 0; j <= nsteps; ++j) {
        PROBE(0);
        if (!tail) {
            if (j < nsteps) {
                // ---- LSTM step j (lstm.c:48-124): row tile = 4 units x gates i, j, f, o
                const int t = b + 2 * j + phase;
                const bool active = valid && t < e;
                v4i bh[2], bl[2];
                load_b<2>(&R.h[cur][0][0], R_STRIDE_, nkt_r, lane, bh, bl);
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
                            const EpRow* er = epl + 16 * rt;
                            int16_t gt[4];
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                const int32_t sx = gxv[k][i];
                                const int32_t hx = (hh[i] << 8) + hl[i];
                                int32_t v;
                                if (ACC32) {
                                    const int32_t x = __builtin_expect(xs_sh != 0, 0) ? shift32(sx, xs_sh) : sx;
                                    v = ep_out<true>(wadd(x, hx), er[i].cst, rsh, lsh);
                                } else {
                                    const int64_t x = __builtin_expect(xs_sh != 0, 0) ? shift64((int64_t)sx, xs_sh)
                                                                                      : (int64_t)sx;
                                    const int64_t pre = x + hx + er[i].cst;
                                    v = sat32(__builtin_expect(lsh > 0, 0) ? shift64(pre, lsh) : (pre >> rsh));
                                }
                                gt[i] = (int16_t)(i == 1 ? act_q15<0>(v, tt) : act_q15<1>(v >> 1, tt));
                            }
                            const int32_t c_old = R.c[sc][u];
                            const int32_t c_new = sat32(((int64_t)gt[0] * gt[1] + (int64_t)gt[2] * c_old) >> 15);
                            const int16_t hv = sat16((act_q15<0>(c_new, tt) * gt[3]) >> 15);
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
            if (!GEN) {   // relu6 (N), relu6 (N), linear (NOUT) -- def_nn*.c layers 2..4
                const NnLayer& L2 = img.L[r.li + 1];
                const NnLayer& L3 = img.L[r.li + 2];
                const NnLayer& L4 = img.L[r.li + 3];
                fc_layer<ACC32, SH::R1, SH::NKR, ACT_RELU6, SH::NW, 2>(
                    L2, W + (L2.a_off - r.a_off), ep + (L2.ep_off - r.ep_lo), in, R_STRIDE_, &R.act[0][0][0],
                    R_STRIDE_, tt, lane);
                wave_lds_sync();
                PROBE(3);
                fc_layer<ACC32, SH::R2, SH::NKR, ACT_RELU6, SH::NW, 2>(
                    L3, W + (L3.a_off - r.a_off), ep + (L3.ep_off - r.ep_lo), &R.act[0][0][0], R_STRIDE_,
                    &R.act[1][0][0], R_STRIDE_, tt, lane);
                wave_lds_sync();
                PROBE(4);
                fc_layer<ACC32, SH::R3, SH::NKR, ACT_LINEAR, SH::NOUT, 2>(
                    L4, W + (L4.a_off - r.a_off), ep + (L4.ep_off - r.ep_lo), &R.act[1][0][0], R_STRIDE_,
                    &R.act[0][0][0], R_STRIDE_, tt, lane);
                wave_lds_sync();
                PROBE(5);
                in = &R.act[0][0][0];
            } else {
                int ab = 0;
                for (int i = r.li + 1; i < img.nl; ++i) {
                    const NnLayer& Ly = img.L[i];
                    int16_t* out = &R.act[ab][0][0];
                    fc_layer<ACC32, 0, 0, -1, 0, 2>(Ly, W + (Ly.a_off - r.a_off), ep + (Ly.ep_off - r.ep_lo), in,
                                                    R_STRIDE_, out, R_STRIDE_, tt, lane);
                    wave_lds_sync();
                    in = out;
                    ab ^= 1;
                }
            }
            // outputs and post-processing (nn_speech.c:92-124)
            const int16_t* fin = in + sc * R_STRIDE_;
            const NnLayer& LO = img.L[img.nl - 1];
            const int nout = GEN ? LO.N : SH::NOUT;
            const bool lin = GEN ? LO.act == ACT_LINEAR : true;
            if (active && r.logits) {
                int32_t* dst = r.logits + ((size_t)s * T + t) * nout;
                for (int o = q; o < nout; o += 4)
                    dst[o] = lin ? reinterpret_cast<const int32_t*>(fin)[o] : (int32_t)fin[o];
            }
            if (lane < 16 && active) {
                if (GEN) {
                    const LogitRow lg = {fin, lin};
                    post_proc(ps, img, lg);
                } else {
                    RegLogits<SH::NOUT> lg;
                    const int32_t* f32 = reinterpret_cast<const int32_t*>(fin);
#pragma unroll
                    for (int o = 0; o < SH::NOUT; ++o) lg.v[o] = f32[o];
                    post_proc(ps, img, lg);
                }
                put_frame(r, s, T, t, ps);
                if (t + 1 < e) put_frame(r, s, T, t + 1, ps);
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
    // ---- feature context (normFeatContext slots 1..5) := last 5 of prev5 ++ feats[b..e):
    // all of the tile's reads before any write (a stream's old slots feed its new ones)
    int4 cv[2];
    int ci[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int idx = g * 64 + lane + 64 * RW * k;   // (stream in tile, 16-byte chunk of 5x40)
        ci[k] = -1;
        if (idx < 16 * 25 && i0 + idx / 25 < nrow) {
            const int st = idx / 25, c = idx - st * 25, m = c / 5, part = c - 5 * m;
            const int L = R.end[st] - R.beg[st];
            if (L > 0) {
                const int gs = sid(i0 + st), j = L + m;
                cv[k] = j < 5 ? *reinterpret_cast<const int4*>(r.prev5 + ((size_t)gs * 5 + j) * 40 + 8 * part)
                              : feat8(r.fs, r.feats, gs, T, R.beg[st], R.beg[st] + j - 5, part);
                ci[k] = gs * 25 + c;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k)
        if (ci[k] >= 0) reinterpret_cast<int4*>(r.prev5)[ci[k]] = cv[k];
}

// ---------------------------------------------------------------------------
// recur_pipe_kernel (the compiled shapes): one 16-stream tile per workgroup of
// LW LSTM waves and 4 tail waves, a 5-stage pipeline across NN steps (S2I: 3
// tail waves, stages 3 and 4 on one):
//   LSTM waves  iteration j: step j   -- Wh.h + gx, gate epilogue, cell and
//                                        hidden update (lstm.c:48-124)
//   tail wave 1 iteration j: step j-1 -- FC relu6  (h  -> a2)
//   tail wave 2 iteration j: step j-2 -- FC relu6  (a2 -> a3)
//   tail wave 3 iteration j: step j-3 -- FC linear (a3 -> logits a4)
//   tail wave 4 iteration j: step j-4 -- outputs, post-processing, trigger
//                                        stores (and the fused controller)
// Only the LSTM stage is recurrent; the other stages hang off it one step
// apart, so a step costs the slowest stage instead of their sum (the
// post-processing alone, 16 lanes of mostly serial work, was as long as an FC
// layer -- profiles/recur_clocks.py).  One workgroup barrier per iteration;
// h, a2, a3 and a4 are double-buffered by iteration parity (stage k reads
// what stage k-1 wrote one iteration earlier, and that buffer is rewritten
// only after the next barrier).
// ---------------------------------------------------------------------------
template <class SH, bool FP = false>
struct PipeCfg {
    // LSTM waves: <= 2 row tiles each (4 tiles each on 4 waves would let KWS's
    // workgroups fit two per CU, but spills ~250 B per lane at 128 VGPRs)
#ifndef PIPE_LW_SMALL
#define PIPE_LW_SMALL 4   // LSTM waves of a net with <= 8 row tiles (VAD's 7)
#endif
    static constexpr int LW = SH::NRT == 0 ? 4 : (SH::NRT <= 8 ? (PIPE_LW_SMALL < SH::NRT ? PIPE_LW_SMALL : SH::NRT) : (SH::NRT + 1) / 2);
    static constexpr int RPW = (SH::NRT + LW - 1) / LW;      // LSTM row tiles per wave
    // the last FC layer and the post-processing on waves of their own (a
    // 5-stage pipeline) for the 2-output nets; S2I keeps them on one wave: a
    // 13th wave would cap the kernel at 128 VGPRs, and the spills cost more
    // than the split gains (profiles/recur_clocks.py)
#ifndef PIPE_S2I_SPLIT
#define PIPE_S2I_SPLIT 0
#endif
    static constexpr int SPLIT = SH::NOUT <= 2 ? 1 : PIPE_S2I_SPLIT;
    // the wide nets' FC stages are as long as the LSTM step: the post wave's
    // frame outputs are stored by the two FC waves (frame t / t + 1) instead of
    // the FC-linear wave
    static constexpr bool STORE_FC12 = SH::NOUT > 2;
    static constexpr int NWV = LW + 3 + SPLIT;               // waves per tile
    // tiles per workgroup (the kernel supports several, sharing the staged
    // weights): one.  Two VAD tiles per workgroup (16 waves, so that every
    // net's recur workgroup fills one CU in a cascade round) measured slower:
    // VAD iteration 2960 -> 4572 cycles with one barrier over both tiles, and
    // no cascade gain (profiles/r02/casc_clocks.py).
    static constexpr int TPW = 1;
    static constexpr int WPG = NWV * TPW;                    // waves per workgroup
    // waves per SIMD the register budget must allow: two workgroups per CU
    // when a workgroup has <= 8 waves (VAD: <= 128 VGPRs), else one
#ifndef PIPE_SMALL_WG_PER_CU
#define PIPE_SMALL_WG_PER_CU 2
#endif
    static constexpr int MINW = SH::NRT <= 8 ? (PIPE_SMALL_WG_PER_CU * WPG + 3) / 4 : (WPG + 3) / 4;
    static_assert(WPG <= 16, "recur_pipe_kernel: at most 16 waves per workgroup");
};

// tiles one workgroup can run back to back through its pipeline (FastRun.tseq)
#define PIPE_KT 4

// the fused prefix stage's LDS (FP): the LSTM input x of a step, per stream
// row the high bytes then the low bytes ^ 0x80 (the B operand's split form),
// rows 16 B longer than the two planes so that the 16 rows of a ds_read_b128
// lane group fall on distinct banks
template <class SH>
struct PipeX {
    static constexpr int XSR = 2 * SH::XS + 16;
};

// KT: tiles the workgroup can hold (PIPE_KT for the multi-tile instantiation,
// else 1); FP: the fused prefix stage's buffers
template <class SH, int KT = PIPE_KT, bool FP = false>
struct alignas(16) PipeTile {
    static constexpr int RS = 64 * SH::NKR + 8;
    static constexpr int CW = cstride(SH::NW);
    int16_t h[2][16][RS];
    int16_t a2[2][16][RS];
    int16_t a3[2][16][RS];
    int16_t a4[2][16][RS];    // stage 3 -> 4: int32 logits
    int16_t hs[KT > 1 ? 16 : 1][RS];   // h at the start of a tile (its LSTM step 0 reads it; several tiles only)
    int32_t c[16][CW];
    // the workgroup's tiles, in pipeline order
    int4 ti[KT][16];          // per stream: {stream, segment begin, end (exclusive), phase | valid << 1}
    int4 ps[KT][16][2];       // PostState (32 bytes) as two 16-byte words
    CascState cst[KT][16];
    int32_t fresh[KT][16];
    int32_t cut[KT][16];      // fused control: frame that reset the net (-1: none)
    int32_t pbt[KT][16];      // frame b of a stream starting at NN phase 1 (no NN, trigger carried), -1: none
    int2 pb[KT][16];          // its outputs: trigger | outputs[0] << 16, outputs[1] | outputs[2] << 16
    // FP: per stream a ring of its last 8 context frames (V index v at slot
    // v & 7), rows 656 B apart: the 16 rows of a B-fragment read fall on
    // distinct banks; and per stream its ring row and the ring slot of V
    // index phase + 4 (pf_load)
    int16_t pfr[FP ? 16 : 1][FP ? 328 : 8];
    int4 pdesc[FP ? 16 : 1];
    // FP: the LSTM input x of three steps (step s in xs[s % 3])
    uint8_t xs[FP ? 3 : 1][FP ? 16 : 1][FP ? PipeX<SH>::XSR : 16];
    int32_t off[8];           // first pipeline step of tiles 1..3 (0x7fffffff past the last), [4]: steps in all
    // the post wave's frame outputs of one step, stored to HBM by another wave
    // one iteration later (double-buffered by iteration parity): frame t,
    // which of t / t + 1 to write (bits 0 / 1), stream, trigger, outputs[3]
    int32_t pt[2][16];
    int32_t pw[2][16];
    int32_t psid[2][16];
    int16_t po[2][16][4];
};
static_assert(PIPE_KT == 4, "the post wave describes one tile per 16 lanes");
static_assert(sizeof(PipeTile<ShapeVad, 1, true>::xs[0]) == 16 * 80, "FP x rows: 80 B");
static_assert(cstride(28) == 30 && cstride(64) == 66 && cstride(72) == 74 && cstride(128) == 130, "cstride");

//
// Fused control (cascade, ca.st non-NULL): the post wave also runs the
// controller (nnCntrlClass_exec) frame by frame as the triggers come out.  At
// the frame that resets the net the stream's segment ends: later frames are
// neither post-processed nor written, the tile's end stores the reset state
// (NNSPClass_reset) instead of the carried one, and the stream is listed for
// its next net -- what casc_control_kernel does after the kernel otherwise.
//
// Several tiles per workgroup (FastRun.tseq, <= PIPE_KT: consecutive 16-entry
// blocks of the stream list) run back to back through ONE pipeline: tile k+1's
// LSTM step 0 follows tile k's last step in the next iteration, while the tail
// stages still drain tile k.  A short segment (a cascade round of 16 frames is
// 8 NN steps) otherwise paid the pipeline's fill and drain -- 4 of every 12
// iterations -- and the weight staging once per tile.  Hand-over at a tile
// boundary:
//   * h: the LSTM waves fetch the next tile's h and c (their own units) at a
//     tile's step 0; h goes to R.hs at step 1 (step 0 of the next tile reads
//     it; step 0 of this one already has), c stays in registers;
//   * the final h, c of a tile: stored to HBM by the LSTM waves at its last
//     step; for a stream whose net was reset (known to the post wave 4
//     iterations later) the FC waves overwrite them with the zero state when
//     they roll the tile's feature context, after an explicit vmcnt(0) wait
//     and a barrier behind the loop;
//   * post-processing and controller state: per tile in LDS (loaded once for
//     all tiles at the start), the post wave switches at the tile's first step
//     and stores the tile's state and bookkeeping at its last.
// Every tile but a workgroup's only one runs at least 2 steps (the hand-overs
// above use a tile's step 1), and every tile at least 1.
// MT: compiled for several tiles (FastRun.tseq > 1).  The one-tile
// instantiation compiles the hand-overs and tile switches away: with them the
// post and LSTM waves' loops carried the switch code (if-converted into
// selects every step), and the FC waves on their SIMDs lost issue slots to it.
template <class SH, bool ACC32, bool MT, bool FP = false>
__global__ __launch_bounds__((64 * PipeCfg<SH, FP>::WPG), (PipeCfg<SH, FP>::MINW)) void recur_pipe_kernel(NnImage img,
                                                                                                    FastRun r,
                                                                                                    CascArgs ca) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    using CF = PipeCfg<SH, FP>;
    using PT = PipeTile<SH, MT ? PIPE_KT : 1, FP>;
    constexpr int KT = MT ? PIPE_KT : 1;
    static_assert(!(FP && MT), "recur_pipe_kernel: the fused prefix stage runs one tile per workgroup");
    constexpr int RGP = CF::LW, RPW = CF::RPW, RS = PT::RS;
    constexpr int N = SH::NW, nrt = SH::NRT, nkt_r = SH::NKR;
    static_assert(CF::TPW == 1, "recur_pipe_kernel: one pipeline per workgroup");
    // the FC stages store their padding rows too (fc_layer<..., PAD>): the
    // rows must fit a stage buffer's row (int32 logits: two int16 each)
    static_assert(16 * SH::R1 <= RS && 16 * SH::R2 <= RS && 32 * SH::R3 <= RS, "padded FC rows exceed RS");
    const bool ctl = ca.st != nullptr;
    // the round after next appends to counts_clear: zero it (every net's recur
    // does; nothing reads or appends to it during this round)
    if (ctl && blockIdx.x == 0 && threadIdx.x < 6) ca.counts_clear[threadIdx.x] = 0;
    const int nrow = r.n_list_dev ? *r.n_list_dev : (r.list ? r.n_list : r.S);
    // (FP: no proj launch records the list length the round ran with)
    if (FP && r.n_list_rec && blockIdx.x == 0 && threadIdx.x == 0) *r.n_list_rec = nrow;
    const int tseq = MT ? r.tseq : 1;   // 1..PIPE_KT (host)
    const int row0 = (int)blockIdx.x * tseq * 16;   // the workgroup's first list entry
    if (row0 >= nrow) return;
    const int nk = MT ? min(tseq, (nrow - row0 + 15) / 16) : 1;   // its tiles
    // development probe (NNSP_RECUR_CLOCKS, the cascade's round 0 / a batch):
    // per workgroup, wall clock (100 MHz) at the start, after staging and at
    // the end, and where it ran (nnsp_hw_where)
    long long* wgc = (NNSP_PROBES && r.dbg_clk && (!ctl || ca.round == 0) && threadIdx.x == 0 && blockIdx.x < 8192u)
                         ? r.dbg_clk + NNSP_DCLK_RECUR + 4 * blockIdx.x
                         : nullptr;
    if (wgc) wgc[0] = (long long)__builtin_amdgcn_s_memrealtime();
    constexpr int TD = 64 * CF::NWV;
    const int tid = (int)threadIdx.x;
    uint8_t* W = smem + TT_BYTES;
    const uint8_t* tt = smem;   // act_q15 tables
    EpRow* ep = reinterpret_cast<EpRow*>(smem + r.a_lds_bytes + TT_BYTES);
    PT& R = *reinterpret_cast<PT*>(smem + r.a_lds_bytes + TT_BYTES + ep_bytes(r.ep_n));
    stage_weights(W, img.A + r.a_off, r.a_lds_bytes);
    stage_ep(ep, img, r.ep_lo, r.ep_n, true, true);
    for (int i = tid; i < TT_BYTES / 16; i += blockDim.x)
        reinterpret_cast<int4*>(smem)[i] = reinterpret_cast<const int4*>(nnsp_tbl_act)[i];
    if (wgc) wgc[1] = (long long)__builtin_amdgcn_s_memrealtime();
    const int lane = tid & 63;
    const int g = __builtin_amdgcn_readfirstlane(tid >> 6);   // < RGP: LSTM wave; then stages
    const int sc = lane & 15, q = lane >> 4;
    auto sid = [&](int i) { return r.list ? r.list[i] : i; };
    const NnLayer& LL = img.L[r.li];
    // compiled shapes have xs_sh == 0 (net_shape): the input and recurrent
    // halves of a gate share one MFMA accumulator
    const int rsh = LL.out_sh < 0 ? -LL.out_sh : 0, lsh = LL.out_sh > 0 ? LL.out_sh : 0;
    const int T = r.T;
    constexpr int SPL = CF::SPLIT;
    const bool post_w = g == RGP + 2 + SPL;   // the post-processing wave
    // the waves that store the post wave's frame outputs one iteration later:
    // the stage with the most slack (FC linear); S2I, whose FC stages are as
    // long as its LSTM step, splits them over its two FC waves (frame t / t + 1)
    constexpr bool SFC = CF::STORE_FC12;
    // (FP: the FC-stage waves' vmcnt(0) would also wait for SFC's output stores)
    static_assert(!(FP && SFC), "recur_pipe_kernel: the fused prefix on nets whose FC stages store outputs");
    const bool store_w = SFC ? (g == RGP || g == RGP + 1) : g == RGP + 2;
    const int store_bits = SFC ? (g == RGP ? 1 : 2) : 3;
    // ---- the tiles' descriptors (post wave, lane = 16 x tile + stream) and
    //      their pipeline steps: the most NN steps of the tile's streams
    if (post_w) {
        const int k = lane >> 4;
        const int i = row0 + 16 * k + sc;
        const bool ok = k < nk && i < nrow;
        const int s = ok ? sid(i) : 0;
        const int b = ok && r.seg_begin ? r.seg_begin[s] : 0;
        const int e = r.seg_len > 0 ? min(T, b + r.seg_len) : T;
        // the post state as two 16-byte words (a PostState copy went
        // through scratch: 2-byte members at odd offsets)
        int4 p0 = make_int4(0, 0, 0, 0), p1 = p0;
        if (ok) {
            p0 = reinterpret_cast<const int4*>(r.post)[2 * s];
            p1 = reinterpret_cast<const int4*>(r.post)[2 * s + 1];
        }
        const int ph = ok ? 1 - (int)(int16_t)(p0.x & 0xffff) : 0;   // 1 - slides
        int m = ok && e - b - ph > 0 ? (e - b - ph + 1) / 2 : 0;
        if (lane < 16) R.pw[0][lane] = R.pw[1][lane] = 0;   // no frame outputs before the first post step
        if (k < KT) {
            R.ti[k][sc] = make_int4(s, b, e, ph | (ok ? 2 : 0));
            R.ps[k][sc][0] = p0;
            R.ps[k][sc][1] = p1;
            R.pbt[k][sc] = -1;
            // fresh[] (frames since the net's reset: the cold front end's frames)
            // as at the kernel start -- the feature-context roll reads through it
            // after the bookkeeping has overwritten it for the next net
            R.fresh[k][sc] = ok && r.fs.nring ? (int)r.fs.fresh[s] : 2;
            if (ctl) {
                CascState cs = {};
                if (ok) cs = ca.st[s];
                R.cst[k][sc] = cs;
            }
        }
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o));
        m = max(m, nk > 1 ? 2 : 1);
        const int m1 = __shfl(m, 16), m2 = __shfl(m, 32), m3 = __shfl(m, 48);
        if (lane == 0) {
            const int o1 = m, o2 = o1 + m1, o3 = o2 + m2, o4 = o3 + m3;
            R.off[1] = nk > 1 ? o1 : 0x7fffffff;
            R.off[2] = nk > 2 ? o2 : 0x7fffffff;
            R.off[3] = nk > 3 ? o3 : 0x7fffffff;
            R.off[4] = nk == 1 ? o1 : (nk == 2 ? o2 : (nk == 3 ? o3 : o4));
        }
    }
    // ---- tile 0's h and c (LSTM waves: the lane's own units); later tiles'
    //      are fetched during the previous tile
    int16_t h_nx[RPW];
    int32_t c_nx[RPW];
    auto fetch_state = [&](int s_, bool ok) {
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            const int u = 4 * (g + RGP * k) + q;
            h_nx[k] = 0;
            c_nx[k] = 0;
            if (g + RGP * k < nrt && u < N) {
                const size_t o = (size_t)(ok ? s_ : 0) * NN_MAX_W + u;
                const int16_t hv = r.h[o];
                const int32_t cv = r.c[o];
                h_nx[k] = ok ? hv : (int16_t)0;
                c_nx[k] = ok ? cv : 0;
            }
        }
    };
    auto put_hs = [&]() {
#pragma unroll
        for (int k = 0; k < RPW; ++k) {
            const int u = 4 * (g + RGP * k) + q;
            if (g + RGP * k < nrt && u < N) R.hs[sc][u] = h_nx[k];
        }
    };
    if (g < RGP) {
        const bool ok = row0 + sc < nrow;
        fetch_state(ok ? sid(row0 + sc) : 0, ok);
        if constexpr (MT) {
            put_hs();
        } else {   // one tile: its step 0 reads h[0] and c as every later step reads them
#pragma unroll
            for (int k = 0; k < RPW; ++k) {
                const int u = 4 * (g + RGP * k) + q;
                if (g + RGP * k < nrt && u < N) {
                    R.h[0][sc][u] = h_nx[k];
                    R.c[sc][u] = c_nx[k];
                }
            }
        }
    }
    __syncthreads();
    const int off1 = __builtin_amdgcn_readfirstlane(R.off[1]);
    const int off2 = __builtin_amdgcn_readfirstlane(R.off[2]);
    const int off3 = __builtin_amdgcn_readfirstlane(R.off[3]);
    const int total = __builtin_amdgcn_readfirstlane(R.off[4]);   // pipeline steps of all tiles
    auto tile_of = [&](int j) { return MT ? (j >= off1 ? 1 : 0) + (j >= off2 ? 1 : 0) + (j >= off3 ? 1 : 0) : 0; };
    auto off_of = [&](int k) { return MT ? (k == 0 ? 0 : (k == 1 ? off1 : (k == 2 ? off2 : off3))) : 0; };
    auto end_of = [&](int k) { return MT && k + 1 < nk ? off_of(k + 1) : total; };
    // staged region: (FP: the layers before the LSTM,) the LSTM's input
    // fragments, then its recurrent ones, then the FC tail
    const uint8_t* Ax = W + (LL.a_off - r.a_off);
    const uint8_t* Ar = W + (LL.ar_off - r.a_off);
    const EpRow* epl = ep + (LL.ep_off - r.ep_lo) + 4 * q;
    // the input half Wx.x of the NEXT step is computed at the end of each
    // step (off the recurrence's critical path) into the accumulators the
    // recurrent half then starts from; its x rows come from proj through HBM
    constexpr int XS = SH::XS;
    v4i axh[RPW], axl[RPW];
    int4 xr[nkt_r][2];
    // The loads land in xr untouched (lanes past the row read column 0 of it)
    // and x_half zeroes those lanes: any use of a load result right after it
    // (a select, a copy) made the wave wait the full load latency every step.
    // the LSTM waves' view of a tile (lane: its stream): first NN frame,
    // segment end, stream, valid -- read from LDS only when a step enters a
    // tile (read every step, the lookup and unpacking cost the LSTM waves VALU
    // issue that the stage waves on their SIMDs then waited for)
    struct TileLane {
        int t0, e, s;
        bool v;
    };
    auto tile_lane = [&](int k) {
        const int4 d = R.ti[k][sc];
        return TileLane{d.y + (d.w & 1), d.z, d.x, (d.w & 2) != 0};
    };
    TileLane ll = {0, 0, 0, false};   // the LSTM step's tile
    TileLane xl = {0, 0, 0, false};   // load_x's tile (xk)
    int xk = -1;
    auto load_x = [&](int jj) {   // split x of pipeline step jj for the lane's stream (B fragments: high, low bytes)
        if constexpr (FP) return;   // (FP: the prefix stage leaves x in R.xs)
        const int kx = tile_of(jj);
        if (MT && kx != xk) {
            xl = tile_lane(kx);
            xk = kx;
        }
        const int jl = jj - off_of(kx);
        const bool ok = xl.v && xl.t0 + 2 * jl < xl.e;
        const uint8_t* src =
            reinterpret_cast<const uint8_t*>(r.xg + ((size_t)(ok ? xl.s : 0) * r.nstep_max + (ok ? jl : 0)) * XS);
#pragma unroll
        for (int kt = 0; kt < nkt_r; ++kt) {
            const int k0 = 64 * kt + 16 * q;
            const uint8_t* p = src + (k0 < XS ? k0 : 0);
            xr[kt][0] = *reinterpret_cast<const int4*>(p);
            xr[kt][1] = *reinterpret_cast<const int4*>(p + XS);
        }
    };
    // ACC32 (int32 accumulators, wrapping): the gate rows' epilogue constants
    // start the low-plane accumulators of the input half, so the gates add
    // nothing but the high plane (mod 2^32 the same sum, affine_acc32b.c's
    // wrap and the proven-int32 acc64 nets alike); the step then loads no cst
    constexpr bool CST_IN_ACC = ACC32;
    // xb (FP): the R.xs slot of the step (step % 3)
    auto x_half = [&](int xb) {   // axh/axl := Wx . x (hi / lo planes) from xr (FP: from R.xs[xb])
        v4i bxh[nkt_r], bxl[nkt_r];
#pragma unroll
        for (int kt = 0; kt < nkt_r; ++kt) {
            // lanes whose k range lies past xs loaded column 0 of the row:
            // used as is, since the A fragments' columns past the LSTM's input
            // width are zero (a select here cost 16 VALU moves per step)
            if constexpr (FP) {
                const int k0 = 64 * kt + 16 * q;
                const uint8_t* xp = &R.xs[xb][sc][k0 < XS ? k0 : 0];
                bxh[kt] = *reinterpret_cast<const v4i*>(xp);
                bxl[kt] = *reinterpret_cast<const v4i*>(xp + XS);
            } else {
                bxh[kt] = v4i{xr[kt][0].x, xr[kt][0].y, xr[kt][0].z, xr[kt][0].w};
                bxl[kt] = v4i{xr[kt][1].x, xr[kt][1].y, xr[kt][1].z, xr[kt][1].w};
            }
        }
#pragma unroll
        for (int k = 0; k < RPW; ++k) {   // one row tile's fragments at a time (no LDS stores here)
            axh[k] = v4i{0, 0, 0, 0};
            axl[k] = v4i{0, 0, 0, 0};
            if (CST_IN_ACC && g + RGP * k < nrt) {
                const EpRow* er = epl + 16 * (g + RGP * k);
                axl[k] = v4i{ep_cst<true>(er[0]), ep_cst<true>(er[1]), ep_cst<true>(er[2]), ep_cst<true>(er[3])};
            }
            if (g + RGP * k < nrt)
#pragma unroll
                for (int kt = 0; kt < nkt_r; ++kt) {
                    const v4i wx = *reinterpret_cast<const v4i*>(Ax + (size_t)((g + RGP * k) * nkt_r + kt) * 1024 + 16 * lane);
                    axh[k] = mfma8(wx, bxh[kt], axh[k]);
                    axl[k] = mfma8(wx, bxl[kt], axl[k]);
                }
        }
    };
    // ---- FP: the prefix stage, on the FC-stage waves RGP and RGP + 1 (row
    //      tiles p, p + 2, ... of the layer before the LSTM: compiled shapes,
    //      one FC layer, K = 240, tanh; the FC stages leave ~1 600 of the
    //      iteration's ~2 500 cycles idle) for step st of the tile's 16
    //      streams, two steps ahead of the LSTM step that reads its output.  Stream k's rows read
    //      the context V[2 st + phase .. + 5] with V = prev5 ++ the segment's
    //      features (as proj_kernel's union, one NN step per MFMA row).  The
    //      frames sit in a per-stream ring of 8 in LDS (R.pfr; V index v at
    //      slot v & 7): a step brings 2 new frames per stream, 160 16-byte
    //      chunks (80 per prefix wave), loaded into registers while the wave
    //      computes the current step and written to the ring behind it, one
    //      barrier before the next step reads them.  The output goes to
    //      R.xs[st % 3] in the LSTM's B-operand form.  No proj launch, and the
    //      x rows do not go through HBM.  (Measured, not kept: the whole 6-frame
    //      window by LDS-DMA per step -- ~380 cycles per global_load_lds issue,
    //      the stage 4 100 cycles against the LSTM's 2 300; one or two
    //      waves of their own -- their chain of k tiles, 5 500 / 3 800 cycles,
    //      and spills at the 96 registers a 9- or 10-wave workgroup allows
    //      twice per CU.)
    const int pfp = g - RGP;   // (FP: 0, 1 on the prefix waves)
    const unsigned prg = (unsigned)r.fs.ring;
    const FeatSrc pfs = r.fs;   // (a copy: a reference into the kernel arguments put them in scratch)
    // the address of V index v of the tile's stream k (the general form:
    // prev5, the ring, the cold frames after a reset; zero row outside a
    // valid stream or past its segment)
    auto pf_src = [&](int k, int v, int part) -> uintptr_t {
        const int4 d = R.ti[0][k];
        const int s_ = d.x, b_ = d.y, e_ = d.z;
        uintptr_t src = reinterpret_cast<uintptr_t>(&nnsp_proj_zero16);
        if (d.w & 2) {
            if (v < 5)
                src = reinterpret_cast<uintptr_t>(r.prev5 + ((size_t)s_ * 5 + v) * 40 + 8 * part);
            else if (b_ + v - 5 < e_)
                src = reinterpret_cast<uintptr_t>(feat8_ptr<true>(pfs, r.feats, s_, T, b_, b_ + v - 5, part,
                                                                  min(max(R.fresh[0][k], 0), 2)));
        }
        return src;
    };
    // this lane's chunk slots of a step's 160 (2 new frames x 16 streams):
    // prefix wave p takes chunks 80 p + lane and 80 p + 64 + lane (lane < 16);
    // chunk c -> stream c / 10, frame (c % 10) / 5 of the two, 8 features
    // c % 5.  (ln: the lane, opaque per use -- hoisted out of the step loop,
    // the per-lane constants pinned ~30 VGPRs and spilled)
    auto pf_chunk = [&](int i, int ln, int& k, int& fw, int& part) {
        const int c = 80 * pfp + ln + 64 * i;
        k = (c * 205) >> 11;   // c / 10 (c < 160)
        const int w = c - 10 * k;
        fw = w >= 5 ? 1 : 0;
        part = w - 5 * fw;
    };
    int4 pf_x[2];   // the staged chunks of the next step's new frames
    // FAST (steps >= 2): the new frames V[2 st + phase + 4, + 5] are past prev5
    // and past the segment's first two (possibly cold) frames -- ring slots
    // (abs0 + b + v - 5 - lookback) mod ring; past the segment they read an
    // in-bounds slot whose rows are not used
    auto pf_load = [&](int st) __attribute__((always_inline)) {
        int ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if (i < 1 || ln < 16) {
                int k, fw, part;
                pf_chunk(i, ln, k, fw, part);
                const int4 pd = R.pdesc[k];   // {row lo, row hi, slot of V index phase + 4, valid}
                unsigned slot = (unsigned)pd.z + (unsigned)(2 * st + fw);
                slot = slot >= prg ? slot - prg : slot;
                const uintptr_t row = (uintptr_t)(uint32_t)pd.x | ((uintptr_t)(uint32_t)pd.y << 32);
                uintptr_t src = pd.w ? row + (uintptr_t)(slot * 80u + 16u * (unsigned)part)
                                     : reinterpret_cast<uintptr_t>(&nnsp_proj_zero16);
                asm volatile("" : "+v"(src));
                pf_x[i] = gload16(src);
            }
        }
    };
    auto pf_store = [&](int st) __attribute__((always_inline)) {   // the staged chunks -> the ring
        int ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            if (i < 1 || ln < 16) {
                int k, fw, part;
                pf_chunk(i, ln, k, fw, part);
                const int v = 2 * st + (R.ti[0][k].w & 1) + 4 + fw;
                *reinterpret_cast<int4*>(&R.pfr[k][(v & 7) * 40 + 8 * part]) = pf_x[i];
            }
        }
    };
    const NnLayer& L0 = img.L[0];
    auto pf_compute = [&](int st, int xb, long long* pp = nullptr) __attribute__((always_inline)) {   // pp: probes
        // B fragments: lane (sc, q), k tile kt = columns 64 kt + 16 q .. + 15 =
        // chunks cc = 8 kt + 2 q and cc + 1 of the 6 x 40 window (chunks 30, 31
        // meet zero A columns: any ring row will do); chunk cc is frame cc / 5,
        // features 8 (cc % 5) .., at V index 2 st + phase + cc / 5
        int qq = q;   // (opaque per step, as in pf_load)
        asm volatile("" : "+v"(qq));
        const int v0 = 2 * st + (R.ti[0][sc].w & 1);
        const int16_t* ring = &R.pfr[sc][0];
        const uint8_t* A0 = W + (L0.a_off - r.a_off);
        const EpRow* e0 = ep + (L0.ep_off - r.ep_lo) + 4 * q;
        const int rsh0 = L0.out_sh < 0 ? -L0.out_sh : 0, lsh0 = L0.out_sh > 0 ? L0.out_sh : 0;
#pragma unroll
        for (int rt = 0; rt < SH::R0; ++rt) {
            if (rt % 2 != pfp) continue;   // this wave's row tiles
            v4i ah = {0, 0, 0, 0};
            // ACC32: the row's constant starts the low-plane accumulator (fc_layer)
            v4i al = ACC32 ? v4i{ep_cst<true>(e0[16 * rt]), ep_cst<true>(e0[16 * rt + 1]), ep_cst<true>(e0[16 * rt + 2]),
                                 ep_cst<true>(e0[16 * rt + 3])}
                           : v4i{0, 0, 0, 0};
            // k tiles two at a time (B 16 VGPRs, A 8): all four at once, with
            // the staged chunks beside them, spilled those right after their
            // loads -- a wait for the load in every step
#pragma unroll
            for (int kh = 0; kh < 2; ++kh) {
                v4i bh[2], bl[2], w[2];
#pragma unroll
                for (int k2 = 0; k2 < 2; ++k2) {
                    const int kt = 2 * kh + k2;
                    int4 h2[2];
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const int cc = 8 * kt + 2 * qq + e;
                        const int f = (cc * 13) >> 6, part = cc - 5 * f;   // cc / 5, cc % 5 (cc < 32)
                        h2[e] = *reinterpret_cast<const int4*>(ring + ((v0 + f) & 7) * 40 + 8 * part);
                    }
                    split_hilo_r(h2[0], h2[1], bh[k2], bl[k2]);
                    w[k2] = *reinterpret_cast<const v4i*>(A0 + (size_t)(rt * 4 + kt) * 1024 + 16 * lane);
                }
#pragma unroll
                for (int k2 = 0; k2 < 2; ++k2) {
                    ah = mfma8(w[k2], bh[k2], ah);
                    al = mfma8(w[k2], bl[k2], al);
                }
                asm volatile("" ::: "memory");
            }
            if (NNSP_PROBES && pp) pp[0] = (long long)__builtin_amdgcn_s_memtime();
            int32_t o[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int32_t acc = (ah[i] << 8) + al[i];
                const int32_t v = ep_out<ACC32>(acc, ACC32 ? 0 : ep_cst<ACC32>(e0[16 * rt + i]), rsh0, lsh0);
                // columns past N: zero (as proj_kernel's x rows; the LSTM's
                // A columns there are zero anyway)
                o[i] = 16 * rt + 4 * q + i < SH::NW ? (int32_t)act16s(ACT_TANH, v, tt) : 0;
            }
            const uint32_t d0 = (uint32_t)(uint16_t)o[0] | ((uint32_t)o[1] << 16);
            const uint32_t d1 = (uint32_t)(uint16_t)o[2] | ((uint32_t)o[3] << 16);
            uint8_t* xp = &R.xs[xb][sc][16 * rt + 4 * q];
            *reinterpret_cast<uint32_t*>(xp) = __builtin_amdgcn_perm(d1, d0, 0x07050301u);
            *reinterpret_cast<uint32_t*>(xp + XS) = __builtin_amdgcn_perm(d1, d0, 0x06040200u) ^ 0x80808080u;
        }
        if (NNSP_PROBES && pp) pp[1] = (long long)__builtin_amdgcn_s_memtime();
    };
    if constexpr (FP) {
        const bool pfw = g == RGP || g == RGP + 1;
        if (pfw) {
            if (pfp == 0 && lane < 16) {   // per stream: its ring row and the slot of V index phase + 4
                const int4 d = R.ti[0][lane];
                const int ph = d.w & 1;
                const int v0 = (pfs.abs0 + d.y + ph + 4 - 5 - pfs.lookback) % (int)prg;
                const uintptr_t row = reinterpret_cast<uintptr_t>(pfs.nring) + (uintptr_t)d.x * prg * 80u;
                R.pdesc[lane] = make_int4((int)(uint32_t)row, (int)(uint32_t)(row >> 32),
                                          v0 < 0 ? v0 + (int)prg : v0, (d.w & 2) ? 1 : 0);
            }
            // V indices phase .. phase + 7 of every stream (the windows of
            // steps 0 and 1) through the general form: 640 chunks, 5 per lane
            // of each prefix wave
            int4 x[5];
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                const int c = 320 * pfp + lane + 64 * i;   // stream c / 40, frame (c % 40) / 5
                const int k = c / 40, w = c - 40 * k, f = w / 5, part = w - 5 * f;
                uintptr_t src = pf_src(k, f + (R.ti[0][k].w & 1), part);
                asm volatile("" : "+v"(src));
                x[i] = gload16(src);
            }
#pragma unroll
            for (int i = 0; i < 5; ++i) {
                const int c = 320 * pfp + lane + 64 * i;
                const int k = c / 40, w = c - 40 * k, f = w / 5, part = w - 5 * f;
                const int v = f + (R.ti[0][k].w & 1);
                *reinterpret_cast<int4*>(&R.pfr[k][(v & 7) * 40 + 8 * part]) = x[i];
            }
        }
        __syncthreads();   // (the ring holds both prefix waves' chunks)
        if (pfw) {
            // steps 0 and 1 before the loop (the LSTM's step 0 reads step 0's
            // x, iteration 0 computes step 1's input half)
            if (total > 2) pf_load(2);
            pf_compute(0, 0);
            asm volatile("" ::: "memory");   // (the two steps one after the other: overlapped, they spilled)
            if (total > 1) pf_compute(1, 1);
        }
        __syncthreads();   // (step 0's window read by both before step 2's frames replace it)
        if (pfw && total > 2) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            pf_store(2);
            if (total > 3) pf_load(3);   // (stored by the loop's first iteration)
        }
        __syncthreads();
    }
    if (g < RGP) {   // (past a segment: row 0 of xg, unused)
        ll = xl = tile_lane(0);
        xk = 0;
        load_x(0);
        x_half(0);
        load_x(1);
    }
    // store the frame outputs the post wave left in slot p (lanes 0..15: the
    // tile's streams)
    auto flush = [&](int p) {   // this wave's share: frame t (store_bits 1), t + 1 (2)
        if (lane < 16) {
            const int fl = R.pw[p][lane] & store_bits;
            if (fl) {
                const int ft = R.pt[p][lane];
                const int fs_ = R.psid[p][lane];
                const int16_t* o = R.po[p][lane];
                if (fl & 1) put_out(r, fs_, T, ft, o[0], o[1], o[2], o[3]);
                if (fl & 2) put_out(r, fs_, T, ft + 1, o[0], o[1], o[2], o[3]);
            }
        }
    };
    // the post wave's state: the current tile's streams (lanes: sc)
    PostState ps = {};
    CascState cst = {};   // fused control: the stream's controller state
    int cut = -1;
    int s = 0, b = 0, e = 0, phase = 0;
    bool valid = false;
    // a tile's first post step: its streams, their post-processing and
    // controller state; frame b of a stream at NN phase 1 (no NN, the trigger
    // carried) runs the controller here, its outputs are stored after the loop
    auto post_start = [&](int tk) {
        const int4 d = R.ti[tk][sc];
        s = d.x;
        b = d.y;
        e = d.z;
        phase = d.w & 1;
        valid = (d.w & 2) != 0;
        cut = -1;
        if (lane < 16) {
            const int4 p0 = R.ps[tk][lane][0], p1 = R.ps[tk][lane][1];
            static_assert(sizeof(PostState) == 32, "PostState: two 16-byte words");
            __builtin_memcpy(&ps, &p0, 16);
            __builtin_memcpy(reinterpret_cast<char*>(&ps) + 16, &p1, 16);
            if (ctl) cst = R.cst[tk][lane];
        }
        if (lane < 16 && valid && phase == 1 && b < e) {
            R.pbt[tk][lane] = b;
            R.pb[tk][lane] =
                make_int2((int)((uint32_t)(uint16_t)ps.trigger | ((uint32_t)(uint16_t)ps.outputs[0] << 16)),
                          (int)((uint32_t)(uint16_t)ps.outputs[1] | ((uint32_t)(uint16_t)ps.outputs[2] << 16)));
            if (ctl && nnsp::casc_step(ca, cst, r.net_id, ps.trigger)) cut = b;
        }
    };
    // a tile's last post step: its post-processing and controller state and
    // reset frame to LDS, for the bookkeeping after the loop (in the loop, its
    // pointers and counters took SGPRs every role's loop then spilled)
    auto post_end = [&](int tk) {
        if (lane < 16) {
            R.cut[tk][lane] = valid ? cut : -1;
            int4 p0, p1;
            __builtin_memcpy(&p0, &ps, 16);
            __builtin_memcpy(&p1, reinterpret_cast<const char*>(&ps) + 16, 16);
            R.ps[tk][lane][0] = p0;
            R.ps[tk][lane][1] = p1;
            R.cst[tk][lane] = cst;
        }
    };
    const NnLayer& L2 = img.L[r.li + 1];
    const NnLayer& L3 = img.L[r.li + 2];
    const NnLayer& L4 = img.L[r.li + 3];
    // development probe (NNSP_RECUR_CLOCKS): s_memtime at the start and end of each
    // iteration's work of LSTM wave 0 and the three stage waves, workgroup 0
    // (RECUR_CLK_WAVE: which LSTM wave records into slots 0-1; development)
#ifndef RECUR_CLK_WAVE
#define RECUR_CLK_WAVE 0
#endif
    constexpr int CLKW = RECUR_CLK_WAVE < RGP ? RECUR_CLK_WAVE : 0;
    long long* clk = (NNSP_PROBES && r.dbg_clk && (!ctl || ca.round == 0) && blockIdx.x == 0 && lane == 0 &&
                      (g == CLKW || g >= RGP))
                         ? r.dbg_clk + 2 * (g == CLKW ? 0 : g - RGP + 1)
                         : nullptr;
    // one pipeline iteration; the buffer parity is a template constant (the
    // loop runs two iterations per trip), so every LDS access of the stages
    // has a constant offset -- indexing the double buffers with a run-time
    // parity cost the S2I post wave ~1100 of its ~6000 cycles per step
    // LSTM wave 0's sub-phases (dbg_clk[1536 + 8 j + k]): loads + MFMA, gates, stores, x_half, load_x
    // (in time order 0, 3, 4, 1, 2)
    long long* lclk = (clk && g == CLKW) ? r.dbg_clk + 1536 : nullptr;
#define LCLK(k) \
    if (lclk && j < 64) lclk[8 * j + (k)] = (long long)__builtin_amdgcn_s_memtime()
    // FP: the prefix stage's share of iteration j (FC-stage waves): step
    // st = j + 2, whose new frames went to the ring in iteration j - 1.  First
    // step st + 1's frames (loaded a whole iteration ago) go to the ring --
    // slots outside step st's window, which the other prefix wave may be
    // reading -- then step st + 2's loads are issued, then step st is
    // computed.  (Loaded at the step and stored after it, the loads were
    // waited for: the HBM latency under load exceeds one step's compute.)
    auto pf_step = [&](const int j) __attribute__((always_inline)) {
        if (j + 2 < total) {
            const int st = j + 2;
            if (st + 1 < total) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the wave's only vector-memory loads: VAD)
                pf_store(st + 1);
            }
            if (st + 2 < total) pf_load(st + 2);
            pf_compute(st, st % 3);
        }
    };
    auto iteration = [&](const int j, auto CUR, auto RL) {
        constexpr int cur = decltype(CUR)::value;
        constexpr int role = decltype(RL)::value;   // 0 LSTM, 1-3 FC stages 1-3, 4 post
        if (clk && j < 64) clk[j * 16] = (long long)__builtin_amdgcn_s_memtime();
        if constexpr (role == 0) {
            if (j < total) {
                // ---- LSTM step j (the tile's step jl): row tile = 4 units x gates i, j, f, o
                const int tk = tile_of(j);
                const int jl = j - off_of(tk);
                const bool first = MT && jl == 0;   // h from R.hs, c from the fetch registers
                if (first) ll = tile_lane(tk);
                const int t = ll.t0 + 2 * jl;
                const bool active = ll.v && t < ll.e;
                const int16_t* hsrc = first ? &R.hs[0][0] : &R.h[cur][0][0];
                v4i bh[nkt_r], bl[nkt_r];
                load_b<nkt_r>(hsrc, RS, nkt_r, lane, bh, bl);
                // every LDS load of the step (A fragments, epilogue constants,
                // cell state, the previous h kept for inactive streams) before
                // the first store: loads cannot be moved across LDS stores
                v4i w[RPW][nkt_r];
                CstT<ACC32> cst[RPW][4];
                int32_t c_old[RPW];
                int16_t h_old[RPW];
#pragma unroll
                for (int k = 0; k < RPW; ++k) {
                    const int rt = g + RGP * k;
                    const int u = 4 * rt + q;
                    c_old[k] = 0;
                    h_old[k] = 0;
                    if (rt < nrt) {
#pragma unroll
                        for (int kt = 0; kt < nkt_r; ++kt)
                            w[k][kt] = *reinterpret_cast<const v4i*>(Ar + (size_t)(rt * nkt_r + kt) * 1024 + 16 * lane);
#pragma unroll
                        for (int i = 0; i < 4; ++i) cst[k][i] = CST_IN_ACC ? 0 : ep_cst<ACC32>(epl[16 * rt + i]);
                        if (u < N) {
                            c_old[k] = first ? c_nx[k] : R.c[sc][u];
                            h_old[k] = hsrc[sc * RS + u];
                        }
                    }
                }
                v4i hh[RPW], hl[RPW];
#pragma unroll
                for (int k = 0; k < RPW; ++k) {
                    hh[k] = axh[k];   // the input half, computed at the end of the previous step
                    hl[k] = axl[k];
                    if (g + RGP * k < nrt)
#pragma unroll
                        for (int kt = 0; kt < nkt_r; ++kt) {
                            hh[k] = mfma8(w[k][kt], bh[kt], hh[k]);
                            hl[k] = mfma8(w[k][kt], bl[kt], hl[k]);
                        }
                }
                LCLK(0);
                // the input half of step j + 1 (axh/axl are free now: consumed
                // above) and the prefetch of x for step j + 2, ahead of the
                // gates: the x_half MFMAs run beside the gates' VALU work and
                // the loads have the gates and stores to land in -- issued at
                // the end of the step, the copy into the loop-carried xr at the
                // loop latch waited out their latency every step
                x_half(FP ? (j + 1) % 3 : 0);
                LCLK(3);
                load_x(j + 2);
                // the next tile's h and c: fetched now, h into R.hs at step 1
                if (MT && first && tk + 1 < nk) {
                    const int4 dn = R.ti[tk + 1][sc];
                    fetch_state(dn.x, (dn.w & 2) != 0);
                }
                LCLK(4);
                int32_t c_new[RPW];
                int16_t hv[RPW];
                // (nolsh: int32 accumulators, no left shift -- as fc_layer)
                const int rsh1 = min(rsh + 1, 31);   // (v >> rsh) >> 1 == v >> min(rsh + 1, 31)
                auto gates = [&](auto nolsh) {
#pragma unroll
                    for (int k = 0; k < RPW; ++k) {
                        const int rt = g + RGP * k;
                        c_new[k] = 0;
                        hv[k] = 0;
                        if (rt < nrt && 4 * rt + q < N) {
                            int16_t gt[4];
#pragma unroll
                            for (int i = 0; i < 4; ++i) {
                                // exact Wx.x + Wh.h (|.| < 2^31 for N <= 128: int32)
                                const int32_t hx = (hh[k][i] << 8) + hl[k][i];
                                int32_t v;
                                if constexpr (decltype(nolsh)::value) {
                                    const int32_t u = wadd(hx, (int32_t)cst[k][i]);
                                    if (i != 1) {   // sigmoid_q15's >> 1 folded into the layer shift
                                        gt[i] = (int16_t)act_q15<1>(u >> rsh1, tt);
                                        continue;
                                    }
                                    v = u >> rsh;
                                } else if (ACC32) {
                                    v = ep_out<true>(hx, cst[k][i], rsh, lsh);
                                } else {
                                    const int64_t pre = (int64_t)hx + cst[k][i];
                                    v = sat32(__builtin_expect(lsh > 0, 0) ? shift64(pre, lsh) : (pre >> rsh));
                                }
                                gt[i] = (int16_t)(i == 1 ? act_q15<0>(v, tt) : act_q15<1>(v >> 1, tt));
                            }
                            c_new[k] = cell_q15_gates(gt[0], gt[1], gt[2], c_old[k]);
                            hv[k] = sat16((act_q15<0>(c_new[k], tt) * gt[3]) >> 15);
                        }
                    }
                };
                if (ACC32 && lsh == 0)
                    gates(std::true_type{});
                else
                    gates(std::false_type{});
                LCLK(1);
                // a tile's last step with another tile behind it: its final
                // state goes to HBM from here (the last tile's: after the loop)
                const bool hand = MT && tk + 1 < nk && j + 1 == off_of(tk + 1) && ll.v;
#pragma unroll
                for (int k = 0; k < RPW; ++k) {
                    const int rt = g + RGP * k;
                    const int u = 4 * rt + q;
                    if (rt < nrt && u < N) {
                        const int32_t cv = active ? c_new[k] : c_old[k];
                        const int16_t hn = active ? hv[k] : h_old[k];
                        R.c[sc][u] = cv;
                        R.h[cur ^ 1][sc][u] = hn;   // h after all groups (T6)
                        if (MT && jl == 1) R.hs[sc][u] = h_nx[k];
                        if (hand) {
                            r.h[(size_t)ll.s * NN_MAX_W + u] = hn;
                            r.c[(size_t)ll.s * NN_MAX_W + u] = cv;
                        }
                    }
                }
                LCLK(2);
            }
        } else if constexpr (role <= 3) {
            if constexpr (FP && role <= 2) pf_step(j);
            if constexpr (role == 1) {   // stage 1: step j-1
                if (j >= 1 && j - 1 < total)
                    fc_layer<ACC32, SH::R1, SH::NKR, ACT_RELU6, SH::NW, SH::NKR, true>(
                        L2, W + (L2.a_off - r.a_off), ep + (L2.ep_off - r.ep_lo), &R.h[cur][0][0], RS, &R.a2[cur][0][0],
                        RS, tt, lane);
                if (SFC) flush(cur ^ 1);
            } else if constexpr (role == 2) {   // stage 2: step j-2
                if (j >= 2 && j - 2 < total)
                    fc_layer<ACC32, SH::R2, SH::NKR, ACT_RELU6, SH::NW, SH::NKR, true>(
                        L3, W + (L3.a_off - r.a_off), ep + (L3.ep_off - r.ep_lo), &R.a2[cur ^ 1][0][0], RS,
                        &R.a3[cur][0][0], RS, tt, lane);
                if (SFC) flush(cur ^ 1);
            } else {   // stage 3 (split): step j-3
                if (j >= 3 && j - 3 < total)
                    fc_layer<ACC32, SH::R3, SH::NKR, ACT_LINEAR, SH::NOUT, SH::NKR, true>(
                        L4, W + (L4.a_off - r.a_off), ep + (L4.ep_off - r.ep_lo), &R.a3[cur ^ 1][0][0], RS,
                        &R.a4[cur][0][0], RS, tt, lane);
                if (!SFC) flush(cur ^ 1);   // the post wave's outputs of the previous iteration
            }
        } else {   // post: step jp = j-3-SPL
          int wfl = 0;   // frames of this step to store (bits: t, t + 1)
          int t = 0;
          const int jp = j - 3 - SPL;
          if (jp >= 0 && jp < total) {
            const int tk = tile_of(jp);
            const int jl = jp - off_of(tk);
            if (MT && jl == 0) post_start(tk);
            t = b + 2 * jl + phase;
            const bool active = valid && t < e;
            if (!SPL) {   // the last FC layer on this wave too
                fc_layer<ACC32, SH::R3, SH::NKR, ACT_LINEAR, SH::NOUT, SH::NKR, true>(
                    L4, W + (L4.a_off - r.a_off), ep + (L4.ep_off - r.ep_lo), &R.a3[cur ^ 1][0][0], RS,
                    &R.a4[cur][0][0], RS, tt, lane);
                wave_lds_sync();
            }
            // outputs and post-processing (nn_speech.c:92-124)
            const int32_t* f32 = reinterpret_cast<const int32_t*>(&R.a4[SPL ? cur ^ 1 : cur][sc][0]);
            if (active && r.logits) {
                int32_t* dst = r.logits + ((size_t)s * T + t) * SH::NOUT;
                for (int o = q; o < SH::NOUT; o += 4) dst[o] = f32[o];
            }
            if (clk && j < 64) clk[j * 16 + 2] = (long long)__builtin_amdgcn_s_memtime();
            if (lane < 16 && active && cut < 0) {
                // logits read from LDS where the post-processing uses them
                // (s2i: 7, and 2 x 17 only on a detection) -- no register copy
                // the 2-output shapes only run with binary post-processing
                // (net_shape, nnsp_batch.c): no s2i path in their loops
                if constexpr (SH::NOUT >= 41) {
                    if (img.nn_id == 0)
                        post_proc_s2i_lds(ps, img, f32);
                    else
                        post_proc(ps, img, LdsLogits{f32});
                } else {
                    post_proc_binary(ps, img, LdsLogits{f32});
                }
            }
            if (clk && j < 64) clk[j * 16 + 3] = (long long)__builtin_amdgcn_s_memtime();
            if (lane < 16 && active && cut < 0) {
                // the controller for frames t and t + 1; their outputs go to
                // the slot, and another wave stores them next iteration (the
                // stores and their address arithmetic off this wave, the
                // pipeline's slowest).  As selects (casc_step_sel): frame t + 1
                // steps the controller only when frame t did not reset the net
                // and t + 1 is inside the segment
                wfl = 1;
                if (ctl) {
                    const bool r0 = nnsp::casc_step_sel(ca, cst, r.net_id, ps.trigger);
                    const CascState c1 = cst;
                    const bool two = !r0 && t + 1 < e;
                    const bool r1 = nnsp::casc_step_sel(ca, cst, r.net_id, ps.trigger);
                    cst = two ? cst : c1;
                    cut = r0 ? t : (two && r1 ? t + 1 : -1);
                    wfl = two ? 3 : 1;
                } else if (t + 1 < e) {
                    wfl = 3;
                }
            }
            if (clk && j < 64) clk[j * 16 + 4] = (long long)__builtin_amdgcn_s_memtime();
          }
          if (lane < 16) {
              R.pw[cur][lane] = wfl;
              if (wfl) {
                  R.pt[cur][lane] = t;
                  R.psid[cur][lane] = s;
                  *reinterpret_cast<int2*>(R.po[cur][lane]) =
                      make_int2((int)((uint32_t)(uint16_t)ps.trigger | ((uint32_t)(uint16_t)ps.outputs[0] << 16)),
                                (int)((uint32_t)(uint16_t)ps.outputs[1] | ((uint32_t)(uint16_t)ps.outputs[2] << 16)));
              }
          }
          // the tile's last step: its post-processing and controller state
          // and reset frame to LDS, for the bookkeeping after the loop (in the
          // loop, its pointers and counters took SGPRs that every role's loop
          // then spilled to VGPR lanes)
          if (MT && jp >= 0 && jp < total) {
              const int tk = tile_of(jp);
              if (jp + 1 == end_of(tk)) post_end(tk);
          }
        }
        if (clk && j < 64) clk[j * 16 + 1] = (long long)__builtin_amdgcn_s_memtime();
        __syncthreads();
    };
    // one loop per wave role (the same trip count, so the same barriers):
    // in one loop over all roles the compiler kept every role's uniform
    // values live across it, spilled ~170 SGPRs to VGPR lanes and paid a
    // v_readlane (a VALU issue) per use -- 15-20 % of the kernel's VALU code
    auto run = [&](auto RL) {
        for (int j = 0; j < total + 3 + SPL; j += 2) {
            iteration(j, std::integral_constant<int, 0>{}, RL);
            if (j + 1 < total + 3 + SPL) iteration(j + 1, std::integral_constant<int, 1>{}, RL);
        }
    };
    if constexpr (!MT)
        if (post_w) post_start(0);
    if (g < RGP)
        run(std::integral_constant<int, 0>{});
    else if (g == RGP)
        run(std::integral_constant<int, 1>{});
    else if (g == RGP + 1)
        run(std::integral_constant<int, 2>{});
    else if (SPL && g == RGP + 2)
        run(std::integral_constant<int, 3>{});
    else
        run(std::integral_constant<int, 4>{});
#undef LCLK
    // the last iteration's post outputs (each iteration ends with a barrier)
    if (store_w) flush((total + 2 + SPL) & 1);
    if constexpr (!MT) {
        if (post_w) post_end(0);
        __syncthreads();
    } else {
        // the earlier tiles' final h / c went out from the LSTM waves at their
        // last step; the zero state of reset streams below must land after
        // them: every wave's stores complete (vmcnt(0)) before the barrier
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    // ---- the tiles' ends, after the loop (inside it, their pointers and
    //      counters cost every role's loop SGPRs, spilled to VGPR lanes).
    //      Frame b of the streams that started at NN phase 1 (no NN, the
    //      trigger carried):
    for (int idx = tid; idx < 16 * nk; idx += TD) {
        const int k = idx >> 4, st = idx & 15;
        const int f = R.pbt[k][st];
        if (f >= 0) {
            const int2 o = R.pb[k][st];
            put_out(r, R.ti[k][st].x, T, f, (int16_t)(o.x & 0xffff), (int16_t)((uint32_t)o.x >> 16),
                    (int16_t)(o.y & 0xffff), (int16_t)((uint32_t)o.y >> 16));
        }
    }
    // LSTM state: the last tile's from LDS (step total-1 wrote h[total & 1]);
    // the earlier tiles' went out from the LSTM waves at their last step.  A
    // stream whose net was reset gets the zero state
    // (NeuralNetClass_setDefault) -- over what the LSTM waves stored, which
    // completed before the barrier above (MT)
    const int tl = nk - 1;
    const int hb = total & 1;
    for (int idx = tid; idx < 16 * N; idx += TD) {
        const int st = idx / N, u = idx - st * N;
        const int4 d = R.ti[tl][st];
        if (d.w & 2) {
            const bool rs = ctl && R.cut[tl][st] >= 0;
            r.h[(size_t)d.x * NN_MAX_W + u] = rs ? (int16_t)0 : R.h[hb][st][u];
            r.c[(size_t)d.x * NN_MAX_W + u] = rs ? 0 : R.c[st][u];
        }
    }
    if (ctl) {
        constexpr int NH = (2 * N + 15) / 16, NC = (4 * N + 15) / 16;   // 16-byte chunks of the h, c rows
        for (int idx = tid; idx < (nk - 1) * 16 * (NH + NC); idx += TD) {
            const int k = idx / (16 * (NH + NC)), rem = idx - k * 16 * (NH + NC);
            const int st = rem / (NH + NC), ch = rem - st * (NH + NC);
            const int4 d = R.ti[k][st];
            if ((d.w & 2) && R.cut[k][st] >= 0) {
                if (ch < NH)
                    reinterpret_cast<int4*>(r.h + (size_t)d.x * NN_MAX_W)[ch] = make_int4(0, 0, 0, 0);
                else
                    reinterpret_cast<int4*>(r.c + (size_t)d.x * NN_MAX_W)[ch - NH] = make_int4(0, 0, 0, 0);
            }
        }
    }
    // ---- feature context (normFeatContext slots 1..5) := last 5 of prev5 ++
    //      feats[b..e); a reset net (FeatureClass_setDefault): slots 1..4 :=
    //      the default, slot 5 := the feature of the frame that reset it (T4).
    //      All reads before any write (a stream's old slots feed its new
    //      ones); every lane loads, through a selected address (selected
    //      values went through scratch)
    auto ctx_src = [&](int idx, int& ci) -> const int4* {   // idx: (tile, stream, 16-byte chunk of 5x40)
        ci = -1;
        const int4* p = &nnsp_proj_zero16;
        const int k = idx / 400, rem = idx - 400 * k;
        if (k < nk) {
            const int st = rem / 25, c = rem - st * 25, m = c / 5, part = c - 5 * m;
            const int4 d = R.ti[k][st];
            const int L = d.z - d.y;
            if ((d.w & 2) && L > 0) {
                const int jx = L + m;
                const int ct = ctl ? R.cut[k][st] : -1;
                const int fr = R.fresh[k][st];
                if (ct >= 0)
                    p = m < 4 ? reinterpret_cast<const int4*>(ca.prev_default[r.net_id]) + part
                              : reinterpret_cast<const int4*>(feat8_ptr<true>(r.fs, r.feats, d.x, T, d.y, ct, part, fr));
                else
                    p = jx < 5 ? reinterpret_cast<const int4*>(r.prev5 + ((size_t)d.x * 5 + jx) * 40 + 8 * part)
                               : reinterpret_cast<const int4*>(
                                     feat8_ptr<true>(r.fs, r.feats, d.x, T, d.y, d.y + jx - 5, part, fr));
                ci = d.x * 25 + c;
            }
        }
        return p;
    };
    constexpr int NCK = (PIPE_KT * 400 + TD - 1) / TD;   // context chunks per thread (named: an array went to scratch)
    static_assert(NCK >= 2 && NCK <= 4, "recur_pipe_kernel: 2-4 context chunks per thread");
    int ci0, ci1, ci2 = -1, ci3 = -1;
    const int4 cv0 = *ctx_src(tid, ci0);
    const int4 cv1 = *ctx_src(tid + TD, ci1);
    int4 cv2 = make_int4(0, 0, 0, 0), cv3 = cv2;
    if constexpr (NCK > 2) cv2 = *ctx_src(tid + 2 * TD, ci2);
    if constexpr (NCK > 3) cv3 = *ctx_src(tid + 3 * TD, ci3);
    __syncthreads();
    int4* p5 = reinterpret_cast<int4*>(r.prev5);
    if (ci0 >= 0) p5[ci0] = cv0;
    if (ci1 >= 0) p5[ci1] = cv1;
    if (ci2 >= 0) p5[ci2] = cv2;
    if (ci3 >= 0) p5[ci3] = cv3;
    // ---- post-processing state and (fused control) the controller's
    //      bookkeeping, casc_control_kernel's tail: frames since the reset of
    //      the net the stream runs next, position, next segment start, next
    //      round's lists.  Post wave, lane = 16 x tile + stream.
    if (post_w) {
        const int k = lane >> 4 < KT ? lane >> 4 : 0;   // (lanes of tiles past KT: not ok below)
        const int4 d = R.ti[k][sc];
        const bool ok = lane >> 4 < nk && (d.w & 2);
        const int sb = d.x, bb = d.y, ee = d.z, ct = R.cut[k][sc];
        if (ok && bb < ee) {
            PostState pz;
            const int4 p0 = R.ps[k][sc][0], p1 = R.ps[k][sc][1];
            __builtin_memcpy(&pz, &p0, 16);
            __builtin_memcpy(reinterpret_cast<char*>(&pz) + 16, &p1, 16);
            if (ct >= 0)
                nnsp::post_reset(pz);
            else
                pz.slides = (int16_t)(pz.slides ^ ((ee - bb) & 1));
            __builtin_memcpy(reinterpret_cast<int4*>(r.post) + 2 * sb, &pz, 32);
        }
        if (ctl) {
            bool want = false;
            int n_next = 0, b_next = T, fr_next = 2;
            if (ok) {
                const CascState cz = R.cst[k][sc];
                fr_next = ct >= 0 ? 0 : min(2, R.fresh[k][sc] + (ee - bb));
                b_next = ct >= 0 ? ct + 1 : ee;
                ca.fresh[sb] = (int8_t)fr_next;
                ca.st[sb] = cz;
                ca.seg_begin[sb] = b_next;
                if (b_next < T) {
                    want = true;
                    n_next = nnsp::seq_at(ca, cz.pos);
                }
            }
            nnsp::list_next(ca, n_next, sb, want, fr_next);
            if (ca.last_round && __ballot(want) && lane == 0) atomicMax(ca.last_round, ca.round + 1);
            nnsp::add_frames(ca, n_next, nnsp::next_frames(ca, T, want, b_next));
            nnsp::count_cuts(ca, ok && ct >= 0);
        }
    }
    if (wgc) {
        wgc[2] = (long long)__builtin_amdgcn_s_memrealtime();
        wgc[3] = (long long)total | (nnsp_hw_where() << 32);
    }
}

// ---------------------------------------------------------------------------
// launch layer
// ---------------------------------------------------------------------------
namespace {

template <class SH>
const void* proj_fn(bool acc32, int gpt) {
    if constexpr (SH::generic) {
        return acc32 ? (const void*)proj_kernel<SH, true, 1> : (const void*)proj_kernel<SH, false, 1>;
    }
    if (gpt == 4) return acc32 ? (const void*)proj_kernel<SH, true, 4> : (const void*)proj_kernel<SH, false, 4>;
    if (gpt == 2) return acc32 ? (const void*)proj_kernel<SH, true, 2> : (const void*)proj_kernel<SH, false, 2>;
    return acc32 ? (const void*)proj_kernel<SH, true, 1> : (const void*)proj_kernel<SH, false, 1>;
}

template <class SH, int RPW>
const void* recur_fn(bool acc32) {
    return acc32 ? (const void*)recur_kernel<SH, RPW, true> : (const void*)recur_kernel<SH, RPW, false>;
}

const void* pick_proj(int shape, bool acc32, int gpt) {
    switch (shape) {
        case NN_SHAPE_VAD: return proj_fn<ShapeVad>(acc32, gpt);
        case NN_SHAPE_KWS: return proj_fn<ShapeKws>(acc32, gpt);
        case NN_SHAPE_S2I: return proj_fn<ShapeS2i>(acc32, gpt);
        default: return proj_fn<ShapeGen>(acc32, gpt);
    }
}

template <class SH>
const void* pipe_fn(bool acc32) {
    return acc32 ? (const void*)recur_pipe_kernel<SH, true, false> : (const void*)recur_pipe_kernel<SH, false, false>;
}
template <class SH>
const void* pipe_fn_mt(bool acc32) {
    return acc32 ? (const void*)recur_pipe_kernel<SH, true, true> : (const void*)recur_pipe_kernel<SH, false, true>;
}
// (int32 accumulators only: the acc64 build spills ~30 VGPRs at the fused
// workgroup's 96-register budget)
template <class SH>
const void* pipe_fn_fp(bool acc32) {
    return acc32 ? (const void*)recur_pipe_kernel<SH, true, false, true> : nullptr;
}

// the shapes with a fused-prefix instantiation (FastRun.fuse): VAD
constexpr bool fuse_shape(int shape) { return shape == NN_SHAPE_VAD; }

// compiled shapes: the pipelined recurrence (one tile per workgroup)
// mode 0: one tile per workgroup; 1: several tiles run back to back
// (FastRun.tseq > 1); 2: one tile, the prefix layers fused in (FastRun.fuse)
template <class SH>
const void* pipe_of(bool acc32, int mode, int* waves, size_t* tile_bytes) {
    if (mode == 2) {
        if constexpr (fuse_shape(std::is_same<SH, ShapeVad>::value ? NN_SHAPE_VAD : NN_SHAPE_GENERIC)) {
            *waves = PipeCfg<SH, true>::WPG;
            *tile_bytes = sizeof(PipeTile<SH, 1, true>);
            return pipe_fn_fp<SH>(acc32);
        }
        return nullptr;
    }
    *waves = PipeCfg<SH>::WPG;
    *tile_bytes = mode == 1 ? sizeof(PipeTile<SH, PIPE_KT>) : sizeof(PipeTile<SH, 1>);
    return mode == 1 ? pipe_fn_mt<SH>(acc32) : pipe_fn<SH>(acc32);
}
const void* pick_pipe(int shape, bool acc32, int* waves, size_t* tile_bytes, int mode = 0) {
    switch (shape) {
        case NN_SHAPE_VAD: return pipe_of<ShapeVad>(acc32, mode, waves, tile_bytes);
        case NN_SHAPE_KWS: return pipe_of<ShapeKws>(acc32, mode, waves, tile_bytes);
        case NN_SHAPE_S2I: return pipe_of<ShapeS2i>(acc32, mode, waves, tile_bytes);
        default: return nullptr;
    }
}

const void* pick_recur(int shape, int nrt, bool acc32) {
    switch (shape) {
        case NN_SHAPE_VAD: return recur_fn<ShapeVad, ShapeVad::RPW>(acc32);
        case NN_SHAPE_KWS: return recur_fn<ShapeKws, ShapeKws::RPW>(acc32);
        case NN_SHAPE_S2I: return recur_fn<ShapeS2i, ShapeS2i::RPW>(acc32);
        default: break;
    }
    const int rpw = (nrt + RG - 1) / RG;
    if (rpw <= 2) return recur_fn<ShapeGen, 2>(acc32);
    if (rpw <= 4) return recur_fn<ShapeGen, 4>(acc32);
    if (rpw <= 5) return recur_fn<ShapeGen, 5>(acc32);
    return recur_fn<ShapeGen, 8>(acc32);
}

int launch(const void* fn, dim3 grid, dim3 blk, size_t lds, void* stream, const NnImage* img, const FastRun* r,
           const CascArgs* ca = nullptr) {
    void* args[3] = {(void*)img, (void*)r, (void*)ca};
    hipError_t e = hipLaunchKernel(fn, grid, blk, args, lds, (hipStream_t)stream);
    return e == hipSuccess ? 0 : (int)e;
}

}  // namespace

extern "C" {

}  // extern "C"

namespace {
template <class SH>
size_t proj_wave_bytes(int gpt) {
    return gpt == 4 ? sizeof(ProjWave<SH, 4>) : (gpt == 2 ? sizeof(ProjWave<SH, 2>) : sizeof(ProjWave<SH, 1>));
}
// gpt: streams per proj tile of the launch (the ProjWave layout depends on it)
// pmode (which 1, compiled shapes): the recurrence instantiation (pick_pipe's
// mode; 1, the largest of the unfused ones, for the planner)
size_t fast_lds_bytes(int which, int a_bytes, int units, int ep_rows, int shape, int gpt, int pmode = 1) {
    // which 0: proj (units = waves); 1: recur (units = tiles per workgroup)
    const size_t base = (size_t)a_bytes + TT_BYTES + ep_bytes(ep_rows);
    size_t pw = sizeof(ProjWave<ShapeGen>), rt = sizeof(RecTile<ShapeGen>);
    int wv = 0;
    switch (shape) {   // compiled shapes: recur runs one pipelined tile per workgroup
        case NN_SHAPE_VAD: pw = proj_wave_bytes<ShapeVad>(gpt); pipe_of<ShapeVad>(false, pmode, &wv, &rt); units = which ? 1 : units; break;
        case NN_SHAPE_KWS: pw = proj_wave_bytes<ShapeKws>(gpt); pipe_of<ShapeKws>(false, pmode, &wv, &rt); units = which ? 1 : units; break;
        case NN_SHAPE_S2I: pw = proj_wave_bytes<ShapeS2i>(gpt); pipe_of<ShapeS2i>(false, pmode, &wv, &rt); units = which ? 1 : units; break;
        default: break;
    }
    return base + (size_t)units * (which == 0 ? pw : rt);
}
}  // namespace

extern "C" {

// the planner's size: proj with one stream per tile (whole-chunk segments)
size_t nnspk_fast_lds_bytes(int which, int a_bytes, int units, int ep_rows, int shape) {
    return fast_lds_bytes(which, a_bytes, units, ep_rows, shape, 1);
}

int nnspk_launch_proj(const NnImage* img, const FastRun* r, int blocks, int waves, void* stream) {
    if (r->shape != NN_SHAPE_GENERIC && r->gpt != 1 && r->gpt != 2 && r->gpt != 4) return (int)hipErrorInvalidValue;
    const size_t lds = fast_lds_bytes(0, r->a_lds_bytes, waves, r->ep_n, r->shape, r->gpt);
    return launch(pick_proj(r->shape, img->acc32 || r->ep32, r->gpt), dim3(blocks), dim3(64 * waves), lds, stream, img, r);
}

int nnspk_fast_fuse_ok(int shape, int a_bytes, int ep_rows, int acc32) {
    return fuse_shape(shape) && acc32 && fast_lds_bytes(1, a_bytes, 1, ep_rows, shape, 1, 2) <= 80 * 1024;
}

int nnspk_launch_recur(const NnImage* img, const FastRun* r, int tpw, const CascArgs_* ctl, void* stream) {
    const int nrow = r->n_list_dev ? r->S : (r->list ? r->n_list : r->S);
    if (nrow <= 0) return 0;
    int waves = 0;
    size_t tb = 0;
    FastRun rr = *r;   // tiles per workgroup, run back to back through its pipeline
    rr.tseq = rr.tseq < 1 ? 1 : (rr.tseq > PIPE_KT ? PIPE_KT : rr.tseq);
    // the fused prefix: one tile per workgroup, features from the cascade's ring
    if (rr.fuse && (!fuse_shape(r->shape) || rr.tseq != 1 || !r->fs.nring || !(img->acc32 || r->ep32)))
        return (int)hipErrorInvalidValue;
    const int pmode = rr.fuse ? 2 : (rr.tseq > 1 ? 1 : 0);
    const size_t lds = r->shape == NN_SHAPE_GENERIC ? nnspk_fast_lds_bytes(1, r->a_lds_bytes, tpw, r->ep_n, r->shape)
                                                    : fast_lds_bytes(1, r->a_lds_bytes, 1, r->ep_n, r->shape, 1, pmode);
    if (const void* fn = pick_pipe(r->shape, img->acc32 || r->ep32, &waves, &tb, pmode)) {
        CascArgs none;
        memset(&none, 0, sizeof none);
        const int tiles = (nrow + 15) / 16;
        return launch(fn, dim3((tiles + rr.tseq - 1) / rr.tseq), dim3(64 * waves), lds, stream, img, &rr,
                      ctl ? ctl : &none);
    }
    if (ctl) return (int)hipErrorInvalidValue;   // fused control needs the pipelined kernel
    const int tiles = (nrow + 15) / 16;
    const int blocks = (tiles + tpw - 1) / tpw;
    return launch(pick_recur(r->shape, img->L[r->li].nrt, img->acc32 || r->ep32), dim3(blocks), dim3(64 * RW * tpw), lds,
                  stream, img, r);
}

int nnspk_set_lds_limit(void) {
    // allow up to 160 KiB of dynamic LDS for every split-path instantiation
    const int shapes[4] = {NN_SHAPE_GENERIC, NN_SHAPE_VAD, NN_SHAPE_KWS, NN_SHAPE_S2I};
    const int nrts[4] = {8, 16, 20, 32};   // one generic recur instantiation each
    for (int a = 0; a < 2; ++a)
        for (int i = 0; i < 4; ++i) {
            int wv = 0;
            size_t tb = 0;
            const void* pipe = pick_pipe(shapes[i], a, &wv, &tb);
            const void* pipe_mt = pick_pipe(shapes[i], a, &wv, &tb, 1);
            const void* pipe_fp = pick_pipe(shapes[i], a, &wv, &tb, 2);
            const void* fns[8] = {pick_proj(shapes[i], a, 1), pick_recur(shapes[i], nrts[i], a),
                                  pick_recur(NN_SHAPE_GENERIC, nrts[i], a), pipe, pick_proj(shapes[i], a, 2),
                                  pick_proj(shapes[i], a, 4), pipe_mt, pipe_fp};
            for (int k = 0; k < 8; ++k) {
                if (!fns[k]) continue;
                hipError_t e = hipFuncSetAttribute(fns[k], hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
                if (e != hipSuccess) return (int)e;
            }
        }
    return 0;
}

}  // extern "C"
