// nnsp_kernels.hip -- hand-written gfx950 kernels of the ns-nnsp hot path and
// the thin C-ABI launch layer the host library calls (nnsp_dev.h has the
// bit-exact building blocks).
//
//   fe_kernel : FeatureClass_execute for every (stream, frame) of a chunk,
//               one wave64 per frame (window, 256-pt radix-4 q31 cFFT with one
//               butterfly per lane, split, power, 40-bank Mel, log10, norm).
//   nn_kernel : NeuralNetClass_exe + NNSPClass post-processing, persistent over
//               the chunk's NN steps; one wave per 16-stream tile; every FC /
//               LSTM matrix product on v_mfma_i32_16x16x64_i8 with int16
//               activations split into hi/lo int8 planes (exact in int32).
//   k_*       : batched single-stage kernels backing the legacy scalar API.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "nnsp_dev.h"
// development probes (s_memtime per phase): compiled in only with -DNNSP_PROBES=1
#ifndef NNSP_PROBES
#define NNSP_PROBES 0
#endif
#include "nnsp_kabi.h"
#include "nnsp_nn.h"

using namespace nnsp;

// development probe (PROBES builds, NnRun.probe): the drop-in kernel's phase
// clocks (s_memrealtime), kept in LDS and written out with the results (a
// store to mapped host memory per phase made each barrier wait for it).
// [0] start, [1] front end done, [2 + i] layer i done, [12] the weight
// staging's end (wave 1), [13] the front end's tables and inputs in, [14]
// post-processing done, [15] results copied out; [16 + 8 i + k] points k
// inside layer i (i < 8; wave 0)
#if NNSP_PROBES
__shared__ long long di_clk[NNSP_PROBE_LONGS];
#define DI_CLK_T(k, tid) \
    do { \
        if (threadIdx.x == (tid)) di_clk[k] = (long long)__builtin_amdgcn_s_memrealtime(); \
    } while (0)
#define DI_CLK(k) \
    do { \
        if (r.probe) DI_CLK_T(k, 0); \
    } while (0)
#else
#define DI_CLK_T(k, tid) do { } while (0)
#define DI_CLK(k) do { } while (0)
#endif

// ============================================================================
// Front end
// ============================================================================
// One wave64 per frame.  The 256-point complex cFFT (arm_radix4_butterfly_q31,
// radix-4 DIF) keeps one butterfly per lane and stage with its four complex
// operands in registers.  Writing a position as c = 64*d3 + 16*d2 + 4*d1 + d0
// (base-4 digits), stage s butterflies over digit d(4-s); register index m is
// that digit and the lane index holds the other three:
//   stage 1  lane = 16*d2 + 4*d1 + d0, m = d3  (loaded straight from the PCM)
//   stage 2  lane = 16*d3 + 4*d1 + d0, m = d2  (T1: m <-> lane bits 4-5, permlane swaps)
//   stage 3  lane = 16*d0 + 4*d3 + d2, m = d1  (T2: through LDS)
//   stage 4  lane = 16*d1 + 4*d3 + d2, m = d0  (T3: permlane swaps)
// The stage-4 outputs go to LDS at their natural bin k = rev8(c) (CMSIS's
// bit reversal), where the split reads bins k and 256-k.  LDS slots are
// swizzled (zslot) so that every one of these accesses is bank-conflict-free.
#define FE_MEL_MAXSEG 3   // max lane segments per Mel bank (nnsp_tbl_melseg)
#define FE_MEL_LEN 11     // MACs per lane segment (tables.mel_segments max_len: 454 coefficients in 62 segments
                          // of <= 11 over the 64 lanes; 12 gave 59, 10 would need 65)
#ifndef FE_WPG
#define FE_WPG 4          // fe_kernel: waves (frames in flight) per workgroup, sharing its LDS tables
                          // (8: one table staging per 8 waves, 37 KB LDS, three workgroups per CU --
                          // measured slower, shared FE 2.19 -> 2.29 ms; profiles/r03/wpg.sh)
#endif
// FE_WPG7=7 (off): the shared front end of the shipped build (72 VGPRs) at
// seven waves per SIMD -- seven-wave workgroups, 36.4 KB LDS, four per CU.
// Measured slower (round 4, paired A/B, 3 runs): shared FE 2.02 -> 2.22 ms,
// cascade 1.158 -> 1.090 G (profiles/r04/fe_seven_waves.jsonl); at 96 % VALU
// issue a seventh wave adds no issue slots, and the bigger workgroups halve
// the turnover the nets' rounds get CUs through.
#ifndef FE_WPG7
#define FE_WPG7 0
#endif
template <int MODE, bool PORT>
struct FeGeom {
    static constexpr bool seven = MODE == 1 /* FE_MODE_SHARED */ && !PORT && FE_WPG7 == 7;
    static constexpr int WPG = seven ? 7 : FE_WPG;     // waves per workgroup
    static constexpr int MINW = seven ? 7 : 6;         // waves per SIMD the registers must allow
    static constexpr int PER_CU = seven ? 4 : 24 / FE_WPG;   // resident workgroups per CU
};
#ifndef FE_PAIR_DEFAULT
#define FE_PAIR_DEFAULT 1   // fe_kernel2 (two frames per wave) for the batch mode
#endif
#define FE_X_DW 512   // dwords of one frame's complex buffer (256 complex)
#define FE_P_DW 260   // dwords of the power spectrum P: bins 0..256 and the Mel segments' zero-coefficient
                      // reads past them (segment start + 11 <= 257; tests/test_tables.py).  fe_kernel's
                      // LDS is 27136 B = 53 x 512 B: six workgroups per CU (LDS is granted in 512-B
                      // blocks -- at 264 the kernel took 27200 B, 54 blocks, five workgroups, -3 %)
__device__ int16_t nnsp_zero_pcm[160];   // input frames before a net's reset (FE_MODE_COLD)
__device__ __forceinline__ int zslot(int c) { return c ^ ((c >> 6) & 2) ^ ((c >> 3) & 4) ^ ((c >> 3) & 8); }

// a wave-uniform offset as such (both halves through readfirstlane): loads
// and stores at base + offset + lane then take the SGPR-base form with a
// 32-bit lane offset, no per-lane 64-bit address arithmetic
__device__ __forceinline__ size_t wave_off(size_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((size_t)hi << 32) | lo;
}
// raw buffer descriptor (stride 0, range 2^31 bytes, CDNA3/4 word 3) on a
// wave-uniform base: loads at a per-lane byte offset with no VALU address math
__device__ __forceinline__ __amdgpu_buffer_rsrc_t pcm_rsrc(const int16_t* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<int16_t*>(base), (short)0, 0x7fffffff, 0x00020000);
}

struct FeLane {
    int mj0, mfirst, mcnt;   // Mel segment start bin; first segment and segment count of bank `lane`
};

// Block-shared constant tables (LDS).
struct FeTables {
    int2 tw[3][3][64];    // per stage, twiddle (k, 2k, 3k) of each lane's butterfly: (cos, sin)
    int4 split[256];      // per bin k: (A_re, A_im, B_re, -) of realCoefA/BQ31 at 16k (PORT: rfft's twiddle)
    int64_t nc[120];      // FE_MODE_SHARED: -mean * stdR of norm[k], norm[120 + k] (fe_kernel's 32-bit path:
                          // (feature - mean) * stdR as one v_mad_i64_i32 of feature, stdR and nc)
    int32_t norm[240];    // FE_MODE_SHARED: k < 120 net k/40's mean of Mel bank k%40, 120 <= k < 240 its
                          // stdR (fe_norm_word) -- dense, so that 40 lanes read 40 banks
    uint32_t logp[128];   // log_tayler_coeff (value, slope) pairs
    uint4 win[64];        // per lane: window taps 128*m + 2*lane, +1 as int16 pairs (0 past tap 479)
    int16_t mc[FE_MEL_LEN][64];   // per lane: its Mel segment's coefficients, zero-padded, read with
                          // sign-extending ds_read_i16 (no VALU unpacking; LDS, not VGPRs:
                          // keeps fe_kernel at 80 VGPRs, six waves per SIMD)
    int8_t bank[64];      // per lane: the bank of its Mel segment (N_MEL = 40: none), read per frame (a
                          // VGPR held across the frame loop cost the batch mode a spill)
};   // 27 KB with fe_kernel's buffers: six workgroups fit the CU's 160 KB
static_assert(sizeof(FeTables) % 16 == 0, "FeTables: copied as 16-byte chunks");
// fe_kernel's LDS (the tables + FE_WPG frame buffers), granted in 512-byte
// blocks, must let 24 / FE_WPG workgroups share a CU's 160 KB: the launch
// bounds (six waves per SIMD) and the grid's generations assume that many
static_assert(((sizeof(FeTables) + FE_WPG * (FE_X_DW + FE_P_DW) * 4 + 511) / 512) * 512 * (24 / FE_WPG) <= 160 * 1024,
              "fe_kernel: LDS per workgroup no longer fits 24 / FE_WPG workgroups per CU");

// the per-net normalisation constants (norm[]; with the Mel pad at 264 the
// tables and buffers stay within 160 KB / 6)
__device__ __forceinline__ int32_t fe_norm_word(const FeArgs& a, int k) {
    if (a.mode != FE_MODE_SHARED || k >= 240) return 0;
    const int n = (k % 120) / 40, b = k % 40;
    if (!a.nring[n]) return 0;
    return k < 120 ? a.nmean[n][b] : a.nstdR[n][b];
}

// ARM_OPTIMIZED=0 (row N4): the tw area holds, per stage and lane, the four
// COMPLEX16 twiddles tw[4k + r] of the lane's butterfly (3 KB of its 4.5 KB)
__device__ __forceinline__ uint4* fe_twp(FeTables& T) { return reinterpret_cast<uint4*>(&T.tw[0][0][0]); }
__device__ __forceinline__ const uint4* fe_twp(const FeTables& T) {
    return reinterpret_cast<const uint4*>(&T.tw[0][0][0]);
}

template <bool PORT>
__device__ __forceinline__ void fe_tables_init(FeTables& T, const FeArgs& a);

// the workgroup's tables: a prebuilt image (FeArgs.tb_img: every load
// independent, one memory latency -- deriving them took ~21 us per workgroup,
// chains of dependent table loads, ~5 % of a front-end workgroup's life) or
// derived in place
// (four 16-byte loads per lane in flight before their stores: with one load
// and its store per iteration a 256-lane workgroup waited four memory
// latencies in a row)
template <bool PORT>
__device__ __forceinline__ void fe_tables_load(FeTables& T, const FeArgs& a) {
    if (a.tb_img) {
        const uint4* src = reinterpret_cast<const uint4*>(a.tb_img);
        uint4* dst = reinterpret_cast<uint4*>(&T);
        constexpr int N = (int)(sizeof(FeTables) / 16);
        const int nt = (int)blockDim.x;
        for (int i0 = threadIdx.x; i0 < N; i0 += 4 * nt) {
            const uint4 v0 = src[i0], v1 = src[min(i0 + nt, N - 1)], v2 = src[min(i0 + 2 * nt, N - 1)],
                        v3 = src[min(i0 + 3 * nt, N - 1)];
            dst[i0] = v0;
            if (i0 + nt < N) dst[i0 + nt] = v1;
            if (i0 + 2 * nt < N) dst[i0 + 2 * nt] = v2;
            if (i0 + 3 * nt < N) dst[i0 + 3 * nt] = v3;
        }
    } else {
        fe_tables_init<PORT>(T, a);
    }
}

// behind the prebuilt tables in FeArgs.tb_img: each lane's Mel segment
// indexes (fe_lane_init's results), read with one vector load per field
// instead of the 64-entry scan of nnsp_tbl_melseg (dependent scalar loads)
struct FeLaneImg {
    int32_t mj0[64], mfirst[64], mcnt[64];
};

template <bool PORT>
__device__ __forceinline__ void fe_tables_init(FeTables& T, const FeArgs& a) {
    if (PORT) {   // fft.c:128-221: stage s butterfly m of its group uses tw[4 m 4^s + r]
        for (int i = threadIdx.x; i < 192; i += blockDim.x) {
            const int s = i / 64, l = i % 64;
            const int k = s == 0 ? l : (s == 1 ? 4 * (l & 15) : 16 * (l >> 4));
            fe_twp(T)[i] = make_uint4((uint32_t)nnsp_tbl_dif_tw[4 * k], (uint32_t)nnsp_tbl_dif_tw[4 * k + 1],
                                      (uint32_t)nnsp_tbl_dif_tw[4 * k + 2], (uint32_t)nnsp_tbl_dif_tw[4 * k + 3]);
        }
        for (int k = threadIdx.x; k < 256; k += blockDim.x)   // rfft's twiddle of bin k (fft.c:103-105)
            T.split[k] = make_int4(nnsp_tbl_dif_rtw[k], 0, 0, 0);
    } else {
        for (int i = threadIdx.x; i < 576; i += blockDim.x) {
            const int s = i / 192, j = (i / 64) % 3, l = i % 64;
            const int k = s == 0 ? l : (s == 1 ? 4 * (l & 15) : 16 * (l >> 4));
            T.tw[s][j][l] = make_int2(nnsp_tbl_tw256[2 * (j + 1) * k], nnsp_tbl_tw256[2 * (j + 1) * k + 1]);
        }
        for (int k = threadIdx.x; k < 256; k += blockDim.x)
            T.split[k] = make_int4(nnsp_tbl_split[3 * k], nnsp_tbl_split[3 * k + 1], nnsp_tbl_split[3 * k + 2], 0);
    }
    for (int k = threadIdx.x; k < 240; k += blockDim.x) T.norm[k] = fe_norm_word(a, k);
    for (int k = threadIdx.x; k < 120; k += blockDim.x) T.nc[k] = -(int64_t)fe_norm_word(a, k) * fe_norm_word(a, 120 + k);
    for (int i = threadIdx.x; i < 128; i += blockDim.x)
        T.logp[i] = (uint32_t)(uint16_t)nnsp_tbl_log[2 * i] | ((uint32_t)(uint16_t)nnsp_tbl_log[2 * i + 1] << 16);
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        uint32_t w[4];
        for (int m = 0; m < 4; ++m) {
            const int i = 128 * m + 2 * lane;
            w[m] = i < 480 ? ((uint32_t)(uint16_t)nnsp_tbl_window[i] | ((uint32_t)(uint16_t)nnsp_tbl_window[i + 1] << 16))
                           : 0u;
        }
        const int* sg = nnsp_tbl_melseg + 4 * lane;
        const int mn = sg[2];
        for (int i = 0; i < FE_MEL_LEN; ++i) T.mc[i][lane] = (int16_t)(i < mn ? nnsp_tbl_mel[sg[3] + i] : 0);
        T.win[lane] = make_uint4(w[0], w[1], w[2], w[3]);
        T.bank[lane] = (int8_t)sg[0];
    }
}

__device__ __forceinline__ Tw3 lds_tw3(const FeTables& T, int s, int lane) {
    Tw3 t;
    const int2 a = T.tw[s][0][lane], b = T.tw[s][1][lane], c = T.tw[s][2][lane];
    t.c1 = a.x; t.s1 = a.y; t.c2 = b.x; t.s2 = b.y; t.c3 = c.x; t.s3 = c.y;
    return t;
}

__device__ __forceinline__ void fe_lane_init(FeLane& L, int lane) {
    L.mj0 = nnsp_tbl_melseg[4 * lane + 1];
    L.mfirst = 0;
    L.mcnt = 0;
    for (int k = 0; k < 64; ++k) {
        const int b = nnsp_tbl_melseg[4 * k];
        if (b == lane && L.mcnt == 0) L.mfirst = k;
        if (b == lane) ++L.mcnt;
    }
}

// feature_module.c:67-73: sat16(((int64)feature - mean) * stdR >> sh).  fast
// (host-proved, nnsp_norm_fits32): the product's shifted value fits int32, so
// one v_mad_i64_i32, the 32 bits at sh and a v_med3 clamp are exact.
__device__ __forceinline__ int16_t fe_norm(int32_t lg, int32_t mn, int32_t sr, int sh, int fast) {
    if (fast) {
        const int32_t v = (int32_t)((uint64_t)mad_i64_i32(wsub(lg, mn), sr, 0) >> sh);
        return (int16_t)min(max(v, -32768), 32767);   // v_med3_i32
    }
    return sat16((((int64_t)lg - mn) * sr) >> sh);
}

// log10 with the (value, slope) table in LDS (fixlog10.c:31-61, bit_frac_in 15)
__device__ __forceinline__ int32_t log10_q15_lds(int32_t x, const uint32_t* logp) {
    if (x == 0) x = 1;
    const uint32_t m = (uint32_t)x & 0x7FFFFFFFu;
    // g = -sh of fixlog10.c (sh = 15 - msb(m), 0 for m = 0), |g| <= 15; x << sh
    // (wrapping) or x >> -sh as one 64-bit shift: the low word of (x:0) >> (32 + g)
    const int g = m ? 16 - __builtin_clz(m) : 0;
    const int32_t y = (int32_t)(((int64_t)x << 32) >> (32 + g));
    int32_t kx = (y - 32768) >> 8;
    const int32_t dx = (y - 32768) & 255;   // = (y - 32768) - (kx << 8), kx before the clamp
    kx = kx < 0 ? 0 : (kx > 127 ? 127 : kx);
    const uint32_t pr = logp[kx];
    // 24-bit multiplies (full rate): |slope| < 2^15, 0 <= dx < 2^8; |v| < 2^16,
    // so v * 0x3796 < 2^31 -- the int64 product of fixlog10.c is exact in 32
    int32_t v = (int32_t)(int16_t)(pr & 0xffff) + (__mul24((int32_t)(int16_t)(pr >> 16), dx) >> 15);
    v = __mul24(v, 0x3796) >> 15;
    return wadd(v, __mul24(0x2688, g));
}

// 4x4 transpose of the register index m with the lane's row (lane bits 4-5):
// v[2m], v[2m+1] = (re, im) of register m.  permlane32_swap exchanges the
// upper half of its first operand with the lower half of its second,
// permlane16_swap the odd rows of the first with the even rows of the second.
__device__ __forceinline__ void xpose_rows(int32_t (&v)[8]) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        auto a = __builtin_amdgcn_permlane32_swap((unsigned)v[0 + p], (unsigned)v[4 + p], false, false);
        auto b = __builtin_amdgcn_permlane32_swap((unsigned)v[2 + p], (unsigned)v[6 + p], false, false);
        auto c = __builtin_amdgcn_permlane16_swap(a[0], b[0], false, false);
        auto d = __builtin_amdgcn_permlane16_swap(a[1], b[1], false, false);
        v[0 + p] = (int32_t)c[0]; v[2 + p] = (int32_t)c[1];
        v[4 + p] = (int32_t)d[0]; v[6 + p] = (int32_t)d[1];
    }
}

// T1 / T3 through LDS instead of permlane swaps (FE_XPOSE_LDS bit 0 / bit 1;
// a v_permlane*_swap costs ~3 VALU issue slots, an LDS round trip none):
//   T1 (stage-1 -> stage-2 layout): position c at slot c + 16 (c >> 6) -- rows
//      of 64 padded to 80 -- conflict-free both ways; needs 320 slots, i.e. X
//      and the P buffer behind it (P is dead during the cFFT)
//   T3 (stage-3 -> stage-4 layout): zslot, as T2 / the final store
#ifndef FE_XPOSE_LDS
#define FE_XPOSE_LDS 0
#endif
__device__ __forceinline__ void xpose_t1_lds(int32_t (&v)[8], int32_t* X, int lane) {
    int2* X2 = reinterpret_cast<int2*>(X);
#pragma unroll
    for (int m = 0; m < 4; ++m) X2[80 * m + lane] = make_int2(v[2 * m], v[2 * m + 1]);
    wave_lds_sync();
    const int rb = 80 * (lane >> 4) + (lane & 15);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int2 p = X2[rb + 16 * m];
        v[2 * m] = p.x; v[2 * m + 1] = p.y;
    }
    wave_lds_sync();
}
__device__ __forceinline__ void xpose_t3_lds(int32_t (&v)[8], int32_t* X, int lane) {
    const int cw = 64 * ((lane >> 2) & 3) + 16 * (lane & 3) + (lane >> 4);
#pragma unroll
    for (int m = 0; m < 4; ++m)
        *reinterpret_cast<int2*>(X + 2 * zslot(cw + 4 * m)) = make_int2(v[2 * m], v[2 * m + 1]);
    wave_lds_sync();
    const int cr = 64 * ((lane >> 2) & 3) + 16 * (lane & 3) + 4 * (lane >> 4);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int2 p = *reinterpret_cast<const int2*>(X + 2 * zslot(cr + m));
        v[2 * m] = p.x; v[2 * m + 1] = p.y;
    }
    wave_lds_sync();
}

// cFFT (arm_radix4_butterfly_q31) of one frame held in v in the stage-1
// layout; leaves the output in X at natural bin order (arm_bitreversal_32).
// PORT: the ARM_OPTIMIZED=0 build's fft() (fft.c:128-221) -- the same DIF
// data flow and output order, unscaled butterflies with Q15 twiddles on all
// four outputs (bfly4_port).
template <bool PORT>
__device__ __forceinline__ void fe_bfly(int32_t (&v)[8], const FeTables& TB, int s, int lane) {
    if (PORT) {
        const uint4 w = fe_twp(TB)[64 * s + lane];
        bfly4_port(v, w.x, w.y, w.z, w.w);
    } else if (s == 0) {
        bfly4<true>(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], lds_tw3(TB, 0, lane));
    } else {
        bfly4<false>(v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], lds_tw3(TB, s, lane));
    }
}

template <bool PORT>
__device__ __forceinline__ void wave_cfft256(int32_t (&v)[8], int32_t* X, const FeTables& TB, int lane) {
    fe_bfly<PORT>(v, TB, 0, lane);
    if (FE_XPOSE_LDS & 1)
        xpose_t1_lds(v, X, lane);
    else
        xpose_rows(v);
    fe_bfly<PORT>(v, TB, 1, lane);
    {   // T2: stage-2 layout out, stage-3 layout in
        const int cw = 64 * (lane >> 4) + (lane & 15);
#pragma unroll
        for (int m = 0; m < 4; ++m)
            *reinterpret_cast<int2*>(X + 2 * zslot(cw + 16 * m)) = make_int2(v[2 * m], v[2 * m + 1]);
        wave_lds_sync();
        const int cr = 64 * ((lane >> 2) & 3) + 16 * (lane & 3) + (lane >> 4);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int2 p = *reinterpret_cast<const int2*>(X + 2 * zslot(cr + 4 * m));
            v[2 * m] = p.x; v[2 * m + 1] = p.y;
        }
    }
    fe_bfly<PORT>(v, TB, 2, lane);
    if (FE_XPOSE_LDS & 2)
        xpose_t3_lds(v, X, lane);
    else
        xpose_rows(v);
    if (PORT)   // last stage: k = 0, tw[0..3]
        bfly4_port(v, (uint32_t)nnsp_tbl_dif_tw[0], (uint32_t)nnsp_tbl_dif_tw[1], (uint32_t)nnsp_tbl_dif_tw[2],
                   (uint32_t)nnsp_tbl_dif_tw[3]);
    else
        bfly4_last(v);
    wave_lds_sync();
    {   // register m is DIF position 64*d3 + 16*d2 + 4*d1 + m; its bin is rev8 of that
        const int c = 64 * ((lane >> 2) & 3) + 16 * (lane & 3) + 4 * (lane >> 4);
#pragma unroll
        for (int m = 0; m < 4; ++m)
            *reinterpret_cast<int2*>(X + 2 * zslot(rev8(c + m))) = make_int2(v[2 * m], v[2 * m + 1]);
    }
    wave_lds_sync();
}

// Split of bin k = lane + 64m from the natural-order cFFT output in X.
// (k = 0 yields a don't-care value; DC / Nyquist come from wave_split_dc.)
// PORT: rfft's split of bin k (fft.c:59-120), k = 0 included.
template <bool PORT>
__device__ __forceinline__ void wave_split_bin(const int32_t* X, const FeTables& TB, int lane, int m,
                                               int32_t& re, int32_t& im) {
    const int k = lane + 64 * m;
    const int4 cf = TB.split[k];
    const int2 zk = *reinterpret_cast<const int2*>(X + 2 * zslot(k));
    const int2 zn = *reinterpret_cast<const int2*>(X + 2 * zslot((256 - k) & 255));
    if (PORT)
        split_bin_port(zk.x, zk.y, zn.x, zn.y, (uint32_t)cf.x, re, im);
    else
        split_bin(zk.x, zk.y, zn.x, zn.y, cf.x, cf.y, cf.z, re, im);
}

// The shipped split of bins k = lane + 64 pr + 1 and 256 - k (pr = 0, 1:
// every bin 1..255 once, bin 128 twice) from one pair of LDS reads.
__device__ __forceinline__ void wave_split_pair(const int32_t* X, const FeTables& TB, int lane, int pr, int& k,
                                                int32_t& re0, int32_t& im0, int32_t& re1, int32_t& im1) {
    k = lane + 64 * pr + 1;
    const int4 cf = TB.split[k];
    const int2 zk = *reinterpret_cast<const int2*>(X + 2 * zslot(k));
    const int2 zn = *reinterpret_cast<const int2*>(X + 2 * zslot(256 - k));
    split_pair(zk.x, zk.y, zn.x, zn.y, cf.x, cf.y, cf.z, re0, im0, re1, im1);
}

// DC and Nyquist bins: (p0 + p1) >> 1, (p0 - p1) >> 1 (arm_split_rfft_q31 tail)
__device__ __forceinline__ void wave_split_dc(const int32_t* X, int32_t& dc, int32_t& nyq) {
    const int2 z0 = *reinterpret_cast<const int2*>(X);
    dc = wadd(z0.x, z0.y) >> 1;
    nyq = wsub(z0.x, z0.y) >> 1;
}

// One frame: window -> rfft -> pspec -> mel -> log10 -> normalise.  Each wave
// runs a contiguous range of frames (consecutive frames of a stream re-read
// two thirds of their window from L1/L2) and prefetches the next frame's PCM.
// (256, 6): at most 80 VGPRs, six waves per SIMD (window and Mel coefficients in LDS)
// One instantiation per mode (FE_MODE_*): the batch and cold modes keep the
// 80-VGPR budget of six waves per SIMD without the shared mode's ring writes.
// PORT: the ARM_OPTIMIZED=0 build's front end (row N4: Frac15 window, fft.c's
// rfft, spec2pspec >> 15; spectrogram_module.c:33-77, feature_module.c:58-60).
// fe_body: the kernel's work on WPG waves (fe_kernel: FeGeom's; the drop-in
// call's fused kernel: eight, or one when it runs out of LDS).  LI (the
// drop-in kernel out of LDS): a's inputs and outputs inside in_dst's buffer
// are used at the same offsets of the LDS image li, where the inputs are
// copied to (one stream, one frame: no history)
// IN: the drop-in call's inputs are copied in first (FeArgs.in_bytes)
template <int MODE, bool PORT, int WPG, bool LI = false, bool IN = LI>
__device__ __forceinline__ void fe_body(FeArgs a, uint8_t* li = nullptr, const int4* ksrc = nullptr) {
    // per wave: the cFFT buffer X (256 complex) and, right behind it, the
    // power spectrum P (257 used; +pad for branch-free Mel reads) -- X and P
    // contiguous so that the padded T1 transpose may use both
    __shared__ __attribute__((aligned(16))) int32_t XPs[WPG][FE_X_DW + FE_P_DW];
    __shared__ __attribute__((aligned(16))) FeTables TB;
    const unsigned nrow = a.n_list_dev ? (unsigned)*a.n_list_dev : (a.list ? (unsigned)a.n_list : (unsigned)a.S);
    const unsigned segW = a.seg_len > 0 && a.seg_len < a.T ? (unsigned)a.seg_len : (unsigned)a.T;
    constexpr bool cold = MODE == FE_MODE_COLD;
    constexpr bool shared = MODE == FE_MODE_SHARED;
    const unsigned W = cold ? (segW < 2u ? segW : 2u) : segW;
    const unsigned nfr = nrow * W;   // host guarantees < 2^31
    const unsigned nw = gridDim.x * (unsigned)WPG;
    const unsigned per = (nfr + nw - 1) / nw;
    // Each wave runs one contiguous frame range.  Guided (shared mode,
    // a.sched == FE_SCHED_GUIDED): the last third of the waves -- dispatched
    // last, in blockIdx order -- run a quarter share each and the others 4/3
    // of one.  With equal shares the launch ended on the last-dispatched
    // waves' whole ranges: ~0.3 ms over which the resident waves ran out one
    // by one (wave timeline, profiles/r05/fe_sched/); the quarter shares fill
    // those slots until the long ranges end, and end within ~0.1 ms.
    // (development: a.sched bits 8-15 the tail waves in twelfths of the grid,
    // 16-23 the share divisor; 0: 4 / 12 and 4)
    const bool guided = shared && (a.sched & 0xff) == FE_SCHED_GUIDED;
    const unsigned g12 = ((unsigned)a.sched >> 8) & 0xffu, gdv = ((unsigned)a.sched >> 16) & 0xffu;
    const unsigned tw = guided ? nw * (g12 ? (g12 < 12u ? g12 : 11u) : 4u) / 12u : 0u, bw = nw - tw;
    const unsigned dv = gdv ? gdv : 4u;
    const unsigned Pb = guided ? (unsigned)(((unsigned long long)dv * nfr + (unsigned long long)dv * bw + tw - 1) /
                                            ((unsigned long long)dv * bw + tw))
                               : per;
    const unsigned Ps = (Pb + dv - 1u) / dv;
    auto range_of = [&](unsigned w, unsigned& b, unsigned& e) {
        const unsigned long long s = w < bw ? (unsigned long long)w * Pb : (unsigned long long)bw * Pb + (unsigned long long)(w - bw) * Ps;
        const unsigned long long t = s + (w < bw ? Pb : Ps);
        b = s < nfr ? (unsigned)s : nfr;
        e = t < nfr ? (unsigned)t : nfr;
    };
    {
        unsigned b0, e0;
        range_of(blockIdx.x * (unsigned)WPG, b0, e0);
        if (b0 >= nfr) return;   // no frame for this workgroup (device-sized lists)
    }
    // development probe (NNSP_RECUR_CLOCKS): per wave, wall clock (100 MHz) at
    // the start, after the tables, at the end, and the frames it ran
    const unsigned wid0 = blockIdx.x * (unsigned)WPG + (threadIdx.x >> 6);
    long long* wclk = (NNSP_PROBES && a.dbg_clk && (threadIdx.x & 63) == 0 && wid0 < 32768u) ? a.dbg_clk + 2048 + 4 * wid0 : nullptr;
    if (wclk) wclk[0] = (long long)__builtin_amdgcn_s_memrealtime();
    // the drop-in call's inputs, from mapped host memory (one workgroup; the
    // waves read them only after the barrier behind the tables, whose loads
    // overlap these)
    // (LI: the rebased pointers; otherwise a's own, as they are -- a local
    // copy of them cost the batch mode's 80-VGPR budget a spill)
#define FE_RB(T, p) reinterpret_cast<T>(li + (reinterpret_cast<const uint8_t*>(p) - reinterpret_cast<const uint8_t*>(a.in_dst)))
    const int16_t* const pcm_li = LI ? FE_RB(const int16_t*, a.pcm) : nullptr;
    const int16_t* const tail_li = LI ? FE_RB(const int16_t*, a.tail) : nullptr;
    int16_t* const feats_li = LI ? FE_RB(int16_t*, a.feats) : nullptr;
    int32_t* const dbg_log_li = LI ? FE_RB(int32_t*, a.dbg_log) : nullptr;
#define FE_P(name) (LI ? name##_li : a.name)
    const int lane = threadIdx.x & 63;
    // the inputs' first two shares, the lanes' Mel indexes and the tables:
    // every load in flight before the first store (one memory latency)
    const int nin = IN ? a.in_bytes / 16 : 0, nt = (int)blockDim.x, tid = (int)threadIdx.x;
    // (ksrc: the inputs passed in the kernel arguments, which the launch
    // writes to device memory -- read from there instead of across PCIe)
    const int4* const isrc = ksrc ? ksrc : reinterpret_cast<const int4*>(a.in_src);
    int4* const idst = reinterpret_cast<int4*>(LI ? li : a.in_dst);
    int4 iv0 = make_int4(0, 0, 0, 0), iv1 = make_int4(0, 0, 0, 0);
    if (tid < nin) iv0 = isrc[tid];
    if (tid + nt < nin) iv1 = isrc[tid + nt];
    FeLane L;
    if (a.tb_img) {
        const FeLaneImg* lg = reinterpret_cast<const FeLaneImg*>(reinterpret_cast<const FeTables*>(a.tb_img) + 1);
        L.mj0 = lg->mj0[lane];
        L.mfirst = lg->mfirst[lane];
        L.mcnt = lg->mcnt[lane];
        fe_tables_load<PORT>(TB, a);
    } else {   // (L derived after the tables: not live across their derivation)
        fe_tables_init<PORT>(TB, a);
        fe_lane_init(L, lane);
    }
    if (tid < nin) idst[tid] = iv0;
    if (tid + nt < nin) idst[tid + nt] = iv1;
    for (int i = tid + 2 * nt; i < nin; i += nt) idst[i] = isrc[i];
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    int32_t* X = XPs[wv];
    int32_t* P = XPs[wv] + FE_X_DW;
    // the Mel partial sums go to X, dead once the split has read it (the next
    // frame's cFFT writes X only after the frame's last wave_lds_sync)
    int64_t* Mp = reinterpret_cast<int64_t*>(X);
    __syncthreads();
    if constexpr (LI) DI_CLK_T(13, 0);
    // (after the barrier: the drop-in call copies them in above)
    const int32_t mean = lane < 40 ? (LI ? FE_RB(const int32_t*, a.mean) : a.mean)[lane] : 0;
    const int32_t stdR = lane < 40 ? (LI ? FE_RB(const int32_t*, a.stdR) : a.stdR)[lane] : 0;
#undef FE_RB
    const unsigned wid = blockIdx.x * (unsigned)WPG + (unsigned)wv;
    unsigned fbeg, fend;
    range_of(wid, fbeg, fend);
    if (wclk) wclk[1] = (long long)__builtin_amdgcn_s_memrealtime();
    // frame f = (row i, k): stream s, segment start b, t = b + k (valid below
    // T); walked incrementally (no per-frame division)
    // t >= lim: nothing to do (past the chunk; COLD: past the segment or not
    // within 2 frames of the reset); z: COLD, input frames before z are zero
    struct Pos { unsigned i, k; int s, b, t, lim, z; };
    // the shared front end runs every stream's whole chunk (no list, no
    // segments, no look-back: the host never sets them for that mode)
    auto row_of = [&](Pos& p) {
        if constexpr (shared) {
            p.s = (int)p.i;
            p.b = 0;
        } else {
            p.s = a.list ? a.list[p.i] : (int)p.i;
            p.b = a.seg_begin ? a.seg_begin[p.s] : 0;
        }
        p.lim = a.T;
        p.z = 0;
        if (cold) {
            const int fr = a.fresh[p.s];
            p.z = p.b - fr;
            p.lim = min(min(a.T, p.b + (int)segW), p.b + 2 - fr);
        }
    };
    auto advance = [&](Pos& p) {
        if (++p.k == W) { p.k = 0; ++p.i; row_of(p); }
        p.t = p.b + (int)p.k;
    };
    // samples of input frame fi (relative to the segment start b: the tail
    // before it; input frame fi - lookback of the chunk, or of the history)
    auto frame_ptr = [&](const Pos& p, int fi) -> const int16_t* {
        if (cold) {
            if (fi < p.z) return nnsp_zero_pcm;
        } else if (fi < p.b) {
            return FE_P(tail) + (size_t)p.s * (a.tail_stride ? (unsigned)a.tail_stride : 320u) + (fi - p.b + 2) * 160;
        }
        if constexpr (shared || LI) return FE_P(pcm) + ((size_t)p.s * a.T + fi) * 160;
        const int x = fi - a.lookback;
        return x >= 0 ? a.pcm + ((size_t)p.s * a.T + x) * 160
                      : a.hist + ((size_t)p.s * a.hist_frames + a.hist_frames + x) * 160;
    };
    // lane's window samples 128*m + 2*lane, +1 of frames t-2, t-1, t
    auto load_frame = [&](const Pos& p, uint32_t (&r)[4]) {
        const int o = 2 * lane;
        const int x0 = shared ? p.t - 2 : p.t - 2 - a.lookback;
        if (!cold && p.t - 2 >= p.b && x0 >= 0) {
            // common case (wave-uniform): frames t-2..t are consecutive in the
            // chunk, so the window is 480 contiguous samples from one pointer
            // buffer loads from a descriptor on the window's first sample (a
            // wave-uniform base, SALU) at the lane's byte offset: no per-lane
            // 64-bit address arithmetic per frame
            const __amdgpu_buffer_rsrc_t rs = pcm_rsrc(FE_P(pcm) + wave_off(((size_t)p.s * a.T + x0) * 160));
            const int vo = 2 * o;
            // (the rows' byte offsets as SGPR offsets: one lane-offset VGPR)
            r[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, vo, 0, 0);
            r[1] = __builtin_amdgcn_raw_buffer_load_b32(rs, vo, 256, 0);
            r[2] = __builtin_amdgcn_raw_buffer_load_b32(rs, vo, 512, 0);
            // lanes 48..63 (taps 480..511, window coefficient 0) load a
            // dummy in-frame word: a select of the value, not of the address,
            // was a register write behind the frame's pending stores
            r[3] = __builtin_amdgcn_raw_buffer_load_b32(rs, lane < 48 ? vo + 768 : vo, 0, 0);
            return;
        }
        const int16_t* p0 = frame_ptr(p, p.t - 2);
        const int16_t* p1 = frame_ptr(p, p.t - 1);
        const int16_t* p2 = frame_ptr(p, p.t);
        r[0] = *reinterpret_cast<const uint32_t*>(p0 + o);
        r[1] = *reinterpret_cast<const uint32_t*>(lane < 16 ? p0 + 128 + o : p1 + o - 32);
        r[2] = *reinterpret_cast<const uint32_t*>(lane < 32 ? p1 + 96 + o : p2 + o - 64);
        r[3] = *reinterpret_cast<const uint32_t*>(lane < 48 ? p2 + 64 + o : p2 + o - 96);
    };
    if (fbeg >= fend) return;
    const unsigned ring0 = shared ? (unsigned)a.abs0 % (unsigned)a.ring : 0u;
    // elements between rings: 3 S ring 40 int16 pass 2^32 at cascade sizes the
    // survey asks for (65 536 streams x T = 1000, 262 144 x T = 200): 64-bit
    const size_t nstride = shared ? (size_t)(unsigned)a.S * (unsigned)a.ring * 40u : 0u;
    Pos nx;
    nx.i = fbeg / W;
    nx.k = fbeg - nx.i * W;
    row_of(nx);
    nx.t = nx.b + (int)nx.k;
    uint32_t raw[4] = {0u, 0u, 0u, 0u};
    if (nx.t < nx.lim) load_frame(nx, raw);
    // The frame's features are stored one frame late, after the next frame's
    // window multiply, and the next window's loads are issued only after that
    // multiply (into the same registers).  On gfx9 vmcnt counts stores as well
    // as loads, and the wait for the window samples cannot count past the
    // frame's conditional stores and loads: issued at the end of a frame, the
    // stores were waited for at the next frame's window (and, with the
    // prefetch issued before the multiply, the prefetch too).  Now everything
    // outstanding at that wait was issued a frame earlier.
    bool pend = false;
    unsigned po = 0;          // output row (shared: ring row s * ring + slot; batch: frame fo)
    uint32_t pv01 = 0u;       // features of nets 0 and 1 (batch: the one feature), int16 pair
    int32_t pv2 = 0;          // shared: net 2's feature
    auto flush = [&]() {
        if (pend && lane < 40) {
            if constexpr (shared) {
                // the host allocates the three rings contiguously (nring[n] =
                // nring[0] + n * nstride): one base pointer live in the loop
                // po = s * ring + slot < 2^31 (nnsp_cascade_create); po * 40
                // does not fit 32 bits past 2^26 ring rows: 64-bit offsets
                int16_t* r0 = a.nring[0] + wave_off((size_t)po * 40u);   // po: the same in every lane
                r0[lane] = (int16_t)(pv01 & 0xffff);
                (r0 + nstride)[lane] = (int16_t)(pv01 >> 16);
                (r0 + 2 * nstride)[lane] = (int16_t)pv2;
            } else {
                FE_P(feats)[(size_t)po * 40 + lane] = (int16_t)(pv01 & 0xffff);
            }
        }
    };
    long long* fclk = (NNSP_PROBES && a.dbg_clk && blockIdx.x == 0 && wv == 0 && lane == 0) ? a.dbg_clk + 1024 : nullptr;
#define FCLK(k) \
    if (fclk && f - fbeg < 64u) fclk[8 * (f - fbeg) + (k)] = (long long)__builtin_amdgcn_s_memtime()
    for (unsigned f = fbeg; f < fend; ++f) {
        FCLK(0);
        const Pos cur = nx;
        if (cur.t >= cur.lim) {   // wave-uniform: nothing to compute, only the next prefetch
            if (f + 1 < fend) {
                advance(nx);
                if (nx.t < nx.lim) load_frame(nx, raw);
            }
            continue;
        }
        const int s = cur.s, t = cur.t;
        if (a.hist_out && t >= a.T - a.hist_frames) {
            // frame t's own 160 samples: raw[2] of lanes 32..63 (samples 0..63),
            // raw[3] of lanes 0..47 (64..159)
            int16_t* h = a.hist_out + ((size_t)s * a.hist_frames + (t - (a.T - a.hist_frames))) * 160;
            if (lane >= 32) *reinterpret_cast<uint32_t*>(h + 2 * lane - 64) = raw[2];
            if (lane < 48) *reinterpret_cast<uint32_t*>(h + 64 + 2 * lane) = raw[3];
        }
        const unsigned fo = (unsigned)s * (unsigned)a.T + (unsigned)t;   // output frame index
        // ---- window (spectrogram_module.c:103-119): x[i] = win[i]*buf[i], Q30;
        // complex c = (x[2c], x[2c+1]), c = 64*m + lane
        int32_t v[8];
        {
            const uint4 w4 = TB.win[lane];
            const uint32_t wn[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                v[2 * m] = (int32_t)(int16_t)(wn[m] & 0xffff) * (int32_t)(int16_t)(raw[m] & 0xffff);
                v[2 * m + 1] = (int32_t)(int16_t)(wn[m] >> 16) * (int32_t)(int16_t)(raw[m] >> 16);
                if (PORT) {   // Frac15 (spectrogram_module.c:64-68)
                    v[2 * m] >>= 15;
                    v[2 * m + 1] >>= 15;
                }
            }
        }
        // pin the products here: sunk past the prefetch (next to their use)
        // they kept the old samples live beside the new ones, and the copy
        // between the two at the loop latch waited for the loads again
        asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]));
        if (f + 1 < fend) {   // prefetch the next frame's window (raw is free now)
            advance(nx);
            if (nx.t < nx.lim) load_frame(nx, raw);
        }
        // the previous frame's features, after the loads: a wait the compiler
        // puts into the prefetch code (path merges) must not cover them
        flush();
        pend = false;
        FCLK(1);
        wave_cfft256<PORT>(v, X, TB, lane);
        FCLK(2);
        // ---- split + power (arm_split_rfft_q31, spec2pspec_arm)
        if (!PORT) {
#pragma unroll
            for (int pr = 0; pr < 2; ++pr) {
                int k;
                int32_t re0, im0, re1, im1;
                wave_split_pair(X, TB, lane, pr, k, re0, im0, re1, im1);
                P[k] = pspec_of(re0, im0);
                P[256 - k] = pspec_of(re1, im1);
                if (MODE == FE_MODE_BATCH && a.dbg_spec) {
                    int32_t* ds = a.dbg_spec + (size_t)fo * 1024;
                    ds[2 * k] = re0; ds[2 * k + 1] = im0;
                    ds[1024 - 2 * k] = re0; ds[1024 - 2 * k + 1] = wsub(0, im0);
                    ds[512 - 2 * k] = re1; ds[512 - 2 * k + 1] = im1;
                    ds[512 + 2 * k] = re1; ds[512 + 2 * k + 1] = wsub(0, im1);
                }
            }
        }
#pragma unroll
        for (int m = 0; m < (PORT ? 4 : 0); ++m) {
            int32_t re, im;
            wave_split_bin<PORT>(X, TB, lane, m, re, im);
            P[lane + 64 * m] = PORT ? pspec15_of(re, im) : pspec_of(re, im);
            if (MODE == FE_MODE_BATCH && a.dbg_spec) {
                int32_t* ds = a.dbg_spec + (size_t)fo * 1024;
                const int k = lane + 64 * m;
                if (PORT) {   // rfft's output: bins 0..256 only
                    ds[2 * k] = re; ds[2 * k + 1] = im;
                } else if (k) {
                    ds[2 * k] = re; ds[2 * k + 1] = im;
                    ds[1024 - 2 * k] = re; ds[1024 - 2 * k + 1] = wsub(0, im);
                }
            }
        }
        if (PORT) {
            if (lane == 0) {   // X(N/2+1) = Xe(1) - Xo(1) (fft.c:122-125); bin 0 came from the loop
                const int2 z0 = *reinterpret_cast<const int2*>(X);
                const int32_t nyq = wsub(wadd(z0.x, z0.x) >> 1, wadd(z0.y, z0.y) >> 1);
                P[256] = pspec15_of(nyq, 0);
                if (MODE == FE_MODE_BATCH && a.dbg_spec) {
                    int32_t* ds = a.dbg_spec + (size_t)fo * 1024;
                    ds[512] = nyq; ds[513] = 0;
                }
            }
        } else if (lane == 0) {
            int32_t dc, nyq;
            wave_split_dc(X, dc, nyq);
            P[0] = pspec_of(dc, 0);
            P[256] = pspec_of(nyq, 0);
            if (MODE == FE_MODE_BATCH && a.dbg_spec) {
                int32_t* ds = a.dbg_spec + (size_t)fo * 1024;
                ds[0] = dc; ds[1] = 0; ds[512] = nyq; ds[513] = 0;
            }
        }
        wave_lds_sync();
        FCLK(3);
        // ---- Mel (melSpecProc.c:6-27): lane segments of <= FE_MEL_LEN MACs
        // (zero-padded), each added into its bank's sum with an LDS atomic
        // (integer addition in any order equals the reference's sequential
        // int64 sum): the tail then reads one sum per bank instead of adding
        // up to FE_MEL_MAXSEG partial sums (address selects and 64-bit adds,
        // ~8 VALU per frame).  The zeroing precedes the atomics in this wave's
        // LDS order; slot 40 takes the lanes without a segment (adding 0).
        {
            if (lane <= 40) Mp[lane] = 0;
            int64_t mac = 0;
#pragma unroll
            for (int i = 0; i < FE_MEL_LEN; ++i) mac = mad_i64_i32((int32_t)TB.mc[i][lane], P[L.mj0 + i], mac);
            atomicAdd(reinterpret_cast<unsigned long long*>(Mp) + TB.bank[lane], (unsigned long long)mac);
        }
        wave_lds_sync();
        FCLK(4);
        // ---- log10 (fixlog10.c:53-61), normalise (feature_module.c:67-73)
        if (lane < 40) {
            const int64_t mac = Mp[lane];   // bank `lane`'s sum
            const int32_t lg = log10_q15_lds(sat32_shr15(mac), TB.logp);
            if (MODE == FE_MODE_BATCH && (LI || a.dbg_log)) FE_P(dbg_log)[(size_t)fo * 40 + lane] = lg;
            if constexpr (shared) {
                // (abs0 + t) % ring with t < T <= ring: one conditional subtract
                unsigned slot = ring0 + (unsigned)t;
                if (slot >= (unsigned)a.ring) slot -= (unsigned)a.ring;
                po = (unsigned)s * (unsigned)a.ring + slot;
                // keep the (mean, stdR) LDS reads here: hoisted out of the frame
                // loop they would pin 6 VGPRs and cost a wave per SIMD
                __asm__ volatile("" ::: "memory");
                // each net's normalisation (feature_module.c:67-73); one
                // wave-uniform branch for the three
                int16_t nv[3];
                if (a.norm32) {   // (lg - mean) * stdR = lg * stdR + nc, exact in 64 bits
#pragma unroll
                    for (int n = 0; n < 3; ++n) {
                        const int32_t sr = TB.norm[120 + 40 * n + lane];
                        const int64_t nc = TB.nc[40 * n + lane];
                        const int32_t v = (int32_t)((uint64_t)mad_i64_i32(lg, sr, nc) >> a.nshift[n]);
                        nv[n] = (int16_t)min(max(v, -32768), 32767);   // v_med3_i32
                    }
                } else {
#pragma unroll
                    for (int n = 0; n < 3; ++n) {
                        const int32_t mn = TB.norm[40 * n + lane], sr = TB.norm[120 + 40 * n + lane];
                        nv[n] = fe_norm(lg, mn, sr, a.nshift[n], 0);
                    }
                }
                pv01 = (uint32_t)(uint16_t)nv[0] | ((uint32_t)(uint16_t)nv[1] << 16);
                pv2 = nv[2];
            } else {
                po = fo;
                pv01 = (uint32_t)(uint16_t)fe_norm(lg, mean, stdR, a.norm_shift, a.norm32);
            }
        }
        pend = true;
        wave_lds_sync();
        FCLK(5);
    }
    flush();
    if (wclk) {
        wclk[2] = (long long)__builtin_amdgcn_s_memrealtime();
        wclk[3] = (long long)(fend - fbeg) | (nnsp_hw_where() << 32);
    }
#undef FCLK
#undef FE_P
}
template <int MODE, bool PORT>
__global__ __launch_bounds__((64 * FeGeom<MODE, PORT>::WPG), (FeGeom<MODE, PORT>::MINW)) void fe_kernel(FeArgs a) {
    fe_body<MODE, PORT, FeGeom<MODE, PORT>::WPG>(a);
}
// ---- two frames per wave (FE_MODE_BATCH / FE_MODE_SHARED) -----------------
// The same per-frame arithmetic as fe_kernel, with two frames' instruction
// streams interleaved stage by stage: each LDS round trip of one frame
// (T2, the split reads, the Mel reads, the bank sums) has the other frame's
// butterflies to issue behind it.  About twice the registers (4 waves per
// SIMD instead of 6: 8 frames in flight instead of 6); per wave the X / P
// buffers of both frames; the Mel partial sums live in the frame's P (dead by
// then).
template <bool PORT>
__device__ __forceinline__ void wave_cfft256x2(int32_t (&va)[8], int32_t (&vb)[8], int32_t* XA, int32_t* XB,
                                               const FeTables& TB, int lane) {
    fe_bfly<PORT>(va, TB, 0, lane);
    fe_bfly<PORT>(vb, TB, 0, lane);
    xpose_rows(va);
    xpose_rows(vb);
    fe_bfly<PORT>(va, TB, 1, lane);
    fe_bfly<PORT>(vb, TB, 1, lane);
    {   // T2 of both frames
        const int cw = 64 * (lane >> 4) + (lane & 15);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            *reinterpret_cast<int2*>(XA + 2 * zslot(cw + 16 * m)) = make_int2(va[2 * m], va[2 * m + 1]);
            *reinterpret_cast<int2*>(XB + 2 * zslot(cw + 16 * m)) = make_int2(vb[2 * m], vb[2 * m + 1]);
        }
        wave_lds_sync();
        const int cr = 64 * ((lane >> 2) & 3) + 16 * (lane & 3) + (lane >> 4);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int2 p = *reinterpret_cast<const int2*>(XA + 2 * zslot(cr + 4 * m));
            const int2 q = *reinterpret_cast<const int2*>(XB + 2 * zslot(cr + 4 * m));
            va[2 * m] = p.x; va[2 * m + 1] = p.y;
            vb[2 * m] = q.x; vb[2 * m + 1] = q.y;
        }
    }
    fe_bfly<PORT>(va, TB, 2, lane);
    fe_bfly<PORT>(vb, TB, 2, lane);
    xpose_rows(va);
    xpose_rows(vb);
    if (PORT) {
        bfly4_port(va, (uint32_t)nnsp_tbl_dif_tw[0], (uint32_t)nnsp_tbl_dif_tw[1], (uint32_t)nnsp_tbl_dif_tw[2],
                   (uint32_t)nnsp_tbl_dif_tw[3]);
        bfly4_port(vb, (uint32_t)nnsp_tbl_dif_tw[0], (uint32_t)nnsp_tbl_dif_tw[1], (uint32_t)nnsp_tbl_dif_tw[2],
                   (uint32_t)nnsp_tbl_dif_tw[3]);
    } else {
        bfly4_last(va);
        bfly4_last(vb);
    }
    wave_lds_sync();
    {
        const int c = 64 * ((lane >> 2) & 3) + 16 * (lane & 3) + 4 * (lane >> 4);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            *reinterpret_cast<int2*>(XA + 2 * zslot(rev8(c + m))) = make_int2(va[2 * m], va[2 * m + 1]);
            *reinterpret_cast<int2*>(XB + 2 * zslot(rev8(c + m))) = make_int2(vb[2 * m], vb[2 * m + 1]);
        }
    }
    wave_lds_sync();
}

template <int MODE, bool PORT>
__global__ __launch_bounds__(256, 4) void fe_kernel2(FeArgs a) {
    static_assert(MODE != FE_MODE_COLD, "the cold front end runs fe_kernel");
    __shared__ __attribute__((aligned(16))) int32_t XPs[4][2][FE_X_DW + FE_P_DW];
    __shared__ __attribute__((aligned(16))) FeTables TB;
    const unsigned nrow = a.n_list_dev ? (unsigned)*a.n_list_dev : (a.list ? (unsigned)a.n_list : (unsigned)a.S);
    const unsigned W = a.seg_len > 0 && a.seg_len < a.T ? (unsigned)a.seg_len : (unsigned)a.T;
    constexpr bool shared = MODE == FE_MODE_SHARED;
    const unsigned nfr = nrow * W;   // host guarantees < 2^31
    const unsigned nw = gridDim.x * 4u;
    const unsigned per = ((nfr + nw - 1) / nw + 1) & ~1u;   // even: whole pairs per wave
    if (blockIdx.x * 4u * per >= nfr) return;
    fe_tables_load<PORT>(TB, a);
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    int32_t* XA = XPs[wv][0];
    int32_t* XB = XPs[wv][1];
    int32_t* PA = XA + FE_X_DW;
    int32_t* PB = XB + FE_X_DW;
    FeLane L;
    fe_lane_init(L, lane);
    const int32_t mean = lane < 40 ? a.mean[lane] : 0;
    const int32_t stdR = lane < 40 ? a.stdR[lane] : 0;
    __syncthreads();
    const unsigned wid = blockIdx.x * 4u + (unsigned)wv;
    const unsigned fbeg = wid * per;
    const unsigned fend = fbeg + per < nfr ? fbeg + per : nfr;
    if (fbeg >= fend) return;
    struct Pos { unsigned i, k; int s, b, t, lim; };
    // the shared front end runs every stream's whole chunk (no list, no
    // segments, no look-back): row i is stream i, b = 0
    auto row_of = [&](Pos& p) {
        if constexpr (shared) {
            p.s = (int)p.i;
            p.b = 0;
        } else {
            p.s = a.list ? a.list[p.i] : (int)p.i;
            p.b = a.seg_begin ? a.seg_begin[p.s] : 0;
        }
        p.lim = a.T;
    };
    auto advance = [&](Pos& p) {
        if (++p.k == W) { p.k = 0; ++p.i; row_of(p); }
        p.t = p.b + (int)p.k;
    };
    auto frame_ptr = [&](const Pos& p, int fi) -> const int16_t* {
        if (fi < p.b)
            return a.tail + (size_t)p.s * (a.tail_stride ? (unsigned)a.tail_stride : 320u) + (fi - p.b + 2) * 160;
        if constexpr (shared) return a.pcm + ((size_t)p.s * a.T + fi) * 160;
        const int x = fi - a.lookback;
        return x >= 0 ? a.pcm + ((size_t)p.s * a.T + x) * 160
                      : a.hist + ((size_t)p.s * a.hist_frames + a.hist_frames + x) * 160;
    };
    auto load_frame = [&](const Pos& p, uint32_t (&r)[4]) {
        const int o = 2 * lane;
        const int x0 = shared ? p.t - 2 : p.t - 2 - a.lookback;
        if (p.t - 2 >= p.b && x0 >= 0) {
            const int16_t* q = a.pcm + wave_off(((size_t)p.s * a.T + x0) * 160) + o;
            r[0] = *reinterpret_cast<const uint32_t*>(q);
            r[1] = *reinterpret_cast<const uint32_t*>(q + 128);
            r[2] = *reinterpret_cast<const uint32_t*>(q + 256);
            r[3] = *reinterpret_cast<const uint32_t*>(q + (lane < 48 ? 384 : 0));
            return;
        }
        const int16_t* p0 = frame_ptr(p, p.t - 2);
        const int16_t* p1 = frame_ptr(p, p.t - 1);
        const int16_t* p2 = frame_ptr(p, p.t);
        r[0] = *reinterpret_cast<const uint32_t*>(p0 + o);
        r[1] = *reinterpret_cast<const uint32_t*>(lane < 16 ? p0 + 128 + o : p1 + o - 32);
        r[2] = *reinterpret_cast<const uint32_t*>(lane < 32 ? p1 + 96 + o : p2 + o - 64);
        r[3] = *reinterpret_cast<const uint32_t*>(lane < 48 ? p2 + 64 + o : p2 + o - 96);
    };
    auto window = [&](const uint32_t (&raw)[4], int32_t (&v)[8]) {
        const uint4 w4 = TB.win[lane];
        const uint32_t wn[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            v[2 * m] = (int32_t)(int16_t)(wn[m] & 0xffff) * (int32_t)(int16_t)(raw[m] & 0xffff);
            v[2 * m + 1] = (int32_t)(int16_t)(wn[m] >> 16) * (int32_t)(int16_t)(raw[m] >> 16);
            if (PORT) {
                v[2 * m] >>= 15;
                v[2 * m + 1] >>= 15;
            }
        }
    };
    auto hist_store = [&](const Pos& p, const uint32_t (&raw)[4]) {
        if (a.hist_out && p.t >= a.T - a.hist_frames) {
            int16_t* h = a.hist_out + ((size_t)p.s * a.hist_frames + (p.t - (a.T - a.hist_frames))) * 160;
            if (lane >= 32) *reinterpret_cast<uint32_t*>(h + 2 * lane - 64) = raw[2];
            if (lane < 48) *reinterpret_cast<uint32_t*>(h + 64 + 2 * lane) = raw[3];
        }
    };
    const unsigned ring0 = shared ? (unsigned)a.abs0 % (unsigned)a.ring : 0u;
    const size_t nstride = shared ? (size_t)(unsigned)a.S * (unsigned)a.ring * 40u : 0u;   // as fe_kernel
    // pending outputs of the previous pair (stored after the next pair's window multiply)
    bool pendA = false, pendB = false;
    unsigned poA = 0, poB = 0;
    uint32_t pvA = 0u, pvB = 0u;
    int32_t p2A = 0, p2B = 0;
    auto flush1 = [&](bool pend, unsigned po, uint32_t pv01, int32_t pv2) {
        if (pend && lane < 40) {
            if constexpr (shared) {
                int16_t* r0 = a.nring[0] + wave_off((size_t)po * 40u);   // po: the same in every lane
                r0[lane] = (int16_t)(pv01 & 0xffff);
                (r0 + nstride)[lane] = (int16_t)(pv01 >> 16);
                (r0 + 2 * nstride)[lane] = (int16_t)pv2;
            } else {
                a.feats[(size_t)po * 40 + lane] = (int16_t)(pv01 & 0xffff);
            }
        }
    };
    // log10 + normalise of one frame (lanes < 40) from its Mel partial sums in Mq
    auto tail = [&](const Pos& p, const int64_t* Mq, unsigned& po, uint32_t& pv01, int32_t& pv2) {
        if (lane < 40) {
            int64_t mac = 0;
#pragma unroll
            for (int k = 0; k < FE_MEL_MAXSEG; ++k)
                if (k < L.mcnt) mac += Mq[L.mfirst + k];
            const int32_t lg = log10_q15_lds(sat32_shr15(mac), TB.logp);
            if constexpr (shared) {
                unsigned slot = ring0 + (unsigned)p.t;
                if (slot >= (unsigned)a.ring) slot -= (unsigned)a.ring;
                po = (unsigned)p.s * (unsigned)a.ring + slot;
                __asm__ volatile("" ::: "memory");
                int16_t nv[3];
#pragma unroll
                for (int n = 0; n < 3; ++n) {
                    const int32_t mn = TB.norm[40 * n + lane], sr = TB.norm[120 + 40 * n + lane];
                    nv[n] = fe_norm(lg, mn, sr, a.nshift[n], a.norm32);
                }
                pv01 = (uint32_t)(uint16_t)nv[0] | ((uint32_t)(uint16_t)nv[1] << 16);
                pv2 = nv[2];
            } else {
                po = (unsigned)p.s * (unsigned)a.T + (unsigned)p.t;
                pv01 = (uint32_t)(uint16_t)fe_norm(lg, mean, stdR, a.norm_shift, a.norm32);
            }
        }
    };
    Pos nA, nB;
    nA.i = fbeg / W;
    nA.k = fbeg - nA.i * W;
    row_of(nA);
    nA.t = nA.b + (int)nA.k;
    nB = nA;
    uint32_t rawA[4] = {0u, 0u, 0u, 0u}, rawB[4] = {0u, 0u, 0u, 0u};
    load_frame(nA, rawA);
    if (fbeg + 1 < fend) {
        advance(nB);
        load_frame(nB, rawB);
    }
    for (unsigned f = fbeg; f < fend; f += 2) {
        const Pos cA = nA, cB = nB;
        const bool hasB = f + 1 < fend;   // wave-uniform
        hist_store(cA, rawA);
        if (hasB) hist_store(cB, rawB);
        int32_t va[8], vb[8];
        window(rawA, va);
        window(rawB, vb);
        asm volatile("" : "+v"(va[0]), "+v"(va[1]), "+v"(va[2]), "+v"(va[3]), "+v"(va[4]), "+v"(va[5]), "+v"(va[6]),
                     "+v"(va[7]));
        asm volatile("" : "+v"(vb[0]), "+v"(vb[1]), "+v"(vb[2]), "+v"(vb[3]), "+v"(vb[4]), "+v"(vb[5]), "+v"(vb[6]),
                     "+v"(vb[7]));
        if (f + 2 < fend) {   // prefetch the next pair
            nA = cB;
            advance(nA);
            load_frame(nA, rawA);
            if (f + 3 < fend) {
                nB = nA;
                advance(nB);
                load_frame(nB, rawB);
            }
        }
        flush1(pendA, poA, pvA, p2A);
        flush1(pendB, poB, pvB, p2B);
        wave_cfft256x2<PORT>(va, vb, XA, XB, TB, lane);
        if (!PORT) {
#pragma unroll
            for (int pr = 0; pr < 2; ++pr) {
                int k;
                int32_t a0, a1, a2, a3, b0, b1, b2, b3;
                wave_split_pair(XA, TB, lane, pr, k, a0, a1, a2, a3);
                wave_split_pair(XB, TB, lane, pr, k, b0, b1, b2, b3);
                PA[k] = pspec_of(a0, a1);
                PA[256 - k] = pspec_of(a2, a3);
                PB[k] = pspec_of(b0, b1);
                PB[256 - k] = pspec_of(b2, b3);
            }
        }
#pragma unroll
        for (int m = 0; m < (PORT ? 4 : 0); ++m) {
            int32_t ra, ia, rb, ib;
            wave_split_bin<PORT>(XA, TB, lane, m, ra, ia);
            wave_split_bin<PORT>(XB, TB, lane, m, rb, ib);
            PA[lane + 64 * m] = PORT ? pspec15_of(ra, ia) : pspec_of(ra, ia);
            PB[lane + 64 * m] = PORT ? pspec15_of(rb, ib) : pspec_of(rb, ib);
        }
        if (lane == 0) {
            if (PORT) {
                const int2 za = *reinterpret_cast<const int2*>(XA), zb = *reinterpret_cast<const int2*>(XB);
                PA[256] = pspec15_of(wsub(wadd(za.x, za.x) >> 1, wadd(za.y, za.y) >> 1), 0);
                PB[256] = pspec15_of(wsub(wadd(zb.x, zb.x) >> 1, wadd(zb.y, zb.y) >> 1), 0);
            } else {
                int32_t dc, nyq;
                wave_split_dc(XA, dc, nyq);
                PA[0] = pspec_of(dc, 0);
                PA[256] = pspec_of(nyq, 0);
                wave_split_dc(XB, dc, nyq);
                PB[0] = pspec_of(dc, 0);
                PB[256] = pspec_of(nyq, 0);
            }
        }
        wave_lds_sync();
        {   // Mel (melSpecProc.c:6-27) of both frames; partial sums into the dead X
            int64_t ma = 0, mb = 0;
#pragma unroll
            for (int i = 0; i < FE_MEL_LEN; ++i) {
                const int32_t c0 = TB.mc[i][lane];
                ma = mad_i64_i32(c0, PA[L.mj0 + i], ma);
                mb = mad_i64_i32(c0, PB[L.mj0 + i], mb);
            }
            reinterpret_cast<int64_t*>(XA)[lane] = ma;
            reinterpret_cast<int64_t*>(XB)[lane] = mb;
        }
        wave_lds_sync();
        tail(cA, reinterpret_cast<const int64_t*>(XA), poA, pvA, p2A);
        tail(cB, reinterpret_cast<const int64_t*>(XB), poB, pvB, p2B);
        pendA = true;
        pendB = hasB;
        wave_lds_sync();
    }
    flush1(pendA, poA, pvA, p2A);
    flush1(pendB, poB, pvB, p2B);
}

// ============================================================================
// NN: generic fc / lstm stack on int8 MFMA (the fused path: any stack the
// reference's NeuralNetClass_exe runs -- widths up to its 300-element
// activation buffers, neural_nets.c:9-10, any number of LSTM layers, each
// layer with its own accumulator width)
// ============================================================================
#define NN_KT (NN_MAX_K / 64)         // k tiles of the widest layer input
#define NN_ASTRIDE (NN_MAX_K + 8)     // int16 per stream row of an activation / h buffer (+pad)

struct alignas(16) NnLds {
    int16_t act[2][16][NN_ASTRIDE];   // layer input / output, ping-pong (the reference's input0/1)
    int16_t h[16][NN_ASTRIDE];        // the current LSTM layer's h (its B operand), staged per step
    int16_t tanh_tbl[384];
    int32_t slides[16];
    int32_t active[16];
};

// Ab: NnImage.A (or its LDS copy, offsets rebased); ws / bs: the image's
// wsum / bias (or their LDS copies).  ONE (the drop-in call: stream 0 is the
// tile's only stream): the accumulators of column 0 (lanes 0, 16, 32, 48, four
// rows each) are spread over lanes 0..15, one row each, so that the epilogue
// -- a long dependent chain per row -- runs once per lane instead of four times
template <bool ONE = false>
__device__ __forceinline__ void fc_layer_mfma(const uint8_t* Ab, const int32_t* ws, const int16_t* bs,
                                              const NnLayer& Ly, const int16_t* in, int16_t* out,
                                              const int16_t* tt, int lane, int rt0, int rstep, int pk = -1) {
    if (pk >= 0) DI_CLK_T(pk, 0);
    // the descriptor's fields in registers, and the epilogue in phases (every
    // row's constants and table entries loaded before its first store): its
    // LDS stores could alias those loads (the drop-in kernel's constants sit
    // in LDS), which serialised one row after another, ~1 us per layer
    const NnLayer L = Ly;
    v4i bh[NN_KT], bl[NN_KT];
    load_b<NN_KT>(in, NN_ASTRIDE, L.nkt, lane, bh, bl);
    if (pk >= 0) DI_CLK_T(pk + 1, 0);
    const int sc = lane & 15, q = lane >> 4;
    const uint8_t* A = Ab + L.a_off;
    for (int rt = rt0; rt < L.nrt; rt += rstep) {
        v4i ah = {0, 0, 0, 0}, al = {0, 0, 0, 0};
#pragma unroll
        for (int kt = 0; kt < NN_KT; ++kt)
            if (kt < L.nkt) {
                const v4i w = load_frag(A + (size_t)(rt * L.nkt + kt) * 1024, lane);
                ah = mfma8(w, bh[kt], ah);
                al = mfma8(w, bl[kt], al);
            }
        if (pk >= 0 && rt == rt0) DI_CLK_T(pk + 2, 0);
        if constexpr (ONE) {
            // lane l < 16 takes row 16 rt + l: accumulator l & 3 of lane 16 (l >> 2)
            int32_t x[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = __builtin_amdgcn_ds_bpermute((lane >> 2) << 6, (ah[i] << 8) + al[i]);
            const int k = lane & 3;
            const int32_t xs = k == 0 ? x[0] : (k == 1 ? x[1] : (k == 2 ? x[2] : x[3]));
            const int row = 16 * rt + lane;
            if (lane < 16) {
                const int32_t v = affine_out(xs + ws[L.ep_off + row], bs[L.ep_off + row], L, L.acc32);
                if (row < L.rows) {
                    if (L.act == ACT_LINEAR)
                        reinterpret_cast<int32_t*>(out)[row] = v;
                    else
                        out[row] = act16(L.act, v, tt);
                }
            }
            if (pk >= 0 && rt == rt0) DI_CLK_T(pk + 3, 0);
            continue;
        }
        // (rows up to 16 * nrt: the constants are padded with zeros)
        const int r0 = 16 * rt + 4 * q;
        int32_t v[4];
        int16_t b[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v[i] = ws[L.ep_off + r0 + i];
            b[i] = bs[L.ep_off + r0 + i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = affine_out((ah[i] << 8) + al[i] + v[i], b[i], L, L.acc32);
        if (L.act == ACT_LINEAR) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (r0 + i < L.rows) reinterpret_cast<int32_t*>(out + sc * NN_ASTRIDE)[r0 + i] = v[i];
        } else {
            int16_t o[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) o[i] = act16(L.act, v[i], tt);
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (r0 + i < L.rows) out[sc * NN_ASTRIDE + r0 + i] = o[i];
        }
        if (pk >= 0 && rt == rt0) DI_CLK_T(pk + 3, 0);
    }
}

// lstm_8x16 (lstm.c:15-214): per 4-unit group, gates i,j,f,o; every group
// reads the previous h (T6).  Rows are re-tiled so that lane group q of row
// tile rt holds gates i,j,f,o of unit 4*rt+q in its 4 accumulator registers.
// h comes staged in hbuf; the cell state row of the lane's stream (cg, NULL
// for a padding stream) stays in HBM: lane (sc, q) owns units 4*rt + q.
__device__ __forceinline__ void lstm_layer_mfma(const uint8_t* Ab, const int32_t* ws, const int32_t* wsr,
                                                const int16_t* bs, const NnLayer& Lg, const int16_t* in,
                                                int16_t* out, const int16_t* hbuf, int32_t* cg, const int16_t* tt,
                                                int lane, bool commit, int rt0, int rstep, int pk = -1) {
    if (pk >= 0) DI_CLK_T(pk, 0);
    const NnLayer Ly = Lg;   // (fields in registers, as fc_layer_mfma)
    v4i bxh[NN_KT], bxl[NN_KT], bhh[NN_KT], bhl[NN_KT];
    load_b<NN_KT>(in, NN_ASTRIDE, Ly.nkt, lane, bxh, bxl);
    load_b<NN_KT>(hbuf, NN_ASTRIDE, Ly.nkt_r, lane, bhh, bhl);
    if (pk >= 0) DI_CLK_T(pk + 1, 0);
    const int sc = lane & 15, q = lane >> 4;
    const uint8_t* A = Ab + Ly.a_off;
    const uint8_t* Ar = Ab + Ly.ar_off;
    const int acc32 = Ly.acc32;
    for (int rt = rt0; rt < Ly.nrt; rt += rstep) {
        v4i xh = {0, 0, 0, 0}, xl = {0, 0, 0, 0}, hh = {0, 0, 0, 0}, hl = {0, 0, 0, 0};
#pragma unroll
        for (int kt = 0; kt < NN_KT; ++kt)
            if (kt < Ly.nkt) {
                const v4i w = load_frag(A + (size_t)(rt * Ly.nkt + kt) * 1024, lane);
                xh = mfma8(w, bxh[kt], xh);
                xl = mfma8(w, bxl[kt], xl);
            }
#pragma unroll
        for (int kt = 0; kt < NN_KT; ++kt)
            if (kt < Ly.nkt_r) {
                const v4i w = load_frag(Ar + (size_t)(rt * Ly.nkt_r + kt) * 1024, lane);
                hh = mfma8(w, bhh[kt], hh);
                hl = mfma8(w, bhl[kt], hl);
            }
        if (pk >= 0 && rt == rt0) DI_CLK_T(pk + 2, 0);
        const int u = 4 * rt + q;
        if (u >= Ly.N) continue;
        int16_t g[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int row = 16 * rt + 4 * q + i;
            const int32_t sx = (xh[i] << 8) + xl[i] + ws[Ly.ep_off + row];
            const int32_t sh = (hh[i] << 8) + hl[i] + wsr[Ly.ep_off + row];
            // rc_Krows_8x16 (affine.c:348-407): x part, shift_64b(qi_rec - qi),
            // then the recurrent part + bias with the is_out epilogue
            int64_t pre;
            if (acc32)
                pre = (int64_t)wadd(shift32(sx, Ly.xs_sh), sh);
            else
                pre = shift64((int64_t)sx, Ly.xs_sh) + (int64_t)sh;
            const int32_t v = affine_out(pre, bs[Ly.ep_off + row], Ly, acc32);
            g[i] = i == 1 ? tanh_q15(v, tt) : sigmoid_q15(v, tt);
        }
        const int32_t c_old = cg ? cg[u] : 0;
        const int32_t c_new = sat32(((int64_t)g[0] * g[1] + (int64_t)g[2] * c_old) >> 15);
        const int16_t hv = sat16(((int32_t)tanh_q15(c_new, tt) * g[3]) >> 15);
        if (commit && cg) cg[u] = c_new;
        out[sc * NN_ASTRIDE + u] = hv;
    }
}

// lstm_layer_mfma for the drop-in call (stream 0 alone): the wave's row tiles
// in rounds of four, tile g of a round in lane group g (lanes 16 g..16 g + 15).
// Each tile's MFMA sums of column 0 go through the wave's 2 x 64-word LDS
// scratch scr (row-major per group), so that lane 16 g + l takes row 16 rt_g +
// l: gate l & 3 of unit 4 rt_g + (l >> 2); the first lane of each quad then
// runs the unit's cell.  One epilogue per round instead of four per tile.
__device__ __forceinline__ void lstm_layer_one(const uint8_t* Ab, const int32_t* ws, const int32_t* wsr,
                                               const int16_t* bs, const NnLayer& Lg, const int16_t* in,
                                               int16_t* out, const int16_t* hbuf, int32_t* cg, const int16_t* tt,
                                               int32_t* scr, int lane, bool commit, int rt0, int rstep,
                                               int pk = -1) {
    if (pk >= 0) DI_CLK_T(pk, 0);
    const NnLayer Ly = Lg;
    v4i bxh[NN_KT], bxl[NN_KT], bhh[NN_KT], bhl[NN_KT];
    load_b<NN_KT>(in, NN_ASTRIDE, Ly.nkt, lane, bxh, bxl);
    load_b<NN_KT>(hbuf, NN_ASTRIDE, Ly.nkt_r, lane, bhh, bhl);
    if (pk >= 0) DI_CLK_T(pk + 1, 0);
    const int sc = lane & 15, q = lane >> 4;
    const uint8_t* A = Ab + Ly.a_off;
    const uint8_t* Ar = Ab + Ly.ar_off;
    const int acc32 = Ly.acc32;
    for (int rb = rt0; rb < Ly.nrt; rb += 4 * rstep) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int rt = rb + g * rstep;
            if (rt >= Ly.nrt) break;   // (wave-uniform)
            v4i xh = {0, 0, 0, 0}, xl = {0, 0, 0, 0}, hh = {0, 0, 0, 0}, hl = {0, 0, 0, 0};
#pragma unroll
            for (int kt = 0; kt < NN_KT; ++kt)
                if (kt < Ly.nkt) {
                    const v4i w = load_frag(A + (size_t)(rt * Ly.nkt + kt) * 1024, lane);
                    xh = mfma8(w, bxh[kt], xh);
                    xl = mfma8(w, bxl[kt], xl);
                }
#pragma unroll
            for (int kt = 0; kt < NN_KT; ++kt)
                if (kt < Ly.nkt_r) {
                    const v4i w = load_frag(Ar + (size_t)(rt * Ly.nkt_r + kt) * 1024, lane);
                    hh = mfma8(w, bhh[kt], hh);
                    hl = mfma8(w, bhl[kt], hl);
                }
            if (sc == 0) {   // column 0: rows 4 q .. 4 q + 3 of tile g
                *reinterpret_cast<int4*>(scr + 16 * g + 4 * q) =
                    make_int4((xh[0] << 8) + xl[0], (xh[1] << 8) + xl[1], (xh[2] << 8) + xl[2], (xh[3] << 8) + xl[3]);
                *reinterpret_cast<int4*>(scr + 64 + 16 * g + 4 * q) =
                    make_int4((hh[0] << 8) + hl[0], (hh[1] << 8) + hl[1], (hh[2] << 8) + hl[2], (hh[3] << 8) + hl[3]);
            }
        }
        if (pk >= 0 && rb == rt0) DI_CLK_T(pk + 2, 0);
        // (the same wave's LDS stores, then loads: in order)
        const int rt = rb + q * rstep;
        const bool ok = rt < Ly.nrt;
        const int row = 16 * rt + sc, k = lane & 3;
        const int rr = ok ? row : 0;   // (constants read in range)
        const int32_t sx = scr[lane] + ws[Ly.ep_off + rr];
        const int32_t sh = scr[64 + lane] + wsr[Ly.ep_off + rr];
        // rc_Krows_8x16 (affine.c:348-407), as lstm_layer_mfma
        int64_t pre;
        if (acc32)
            pre = (int64_t)wadd(shift32(sx, Ly.xs_sh), sh);
        else
            pre = shift64((int64_t)sx, Ly.xs_sh) + (int64_t)sh;
        const int32_t v = affine_out(pre, bs[Ly.ep_off + rr], Ly, acc32);
        const int32_t gk = k == 1 ? tanh_q15(v, tt) : sigmoid_q15(v, tt);
        const int qb = (lane & ~3) << 2;   // the quad's first lane
        const int32_t g0 = __builtin_amdgcn_ds_bpermute(qb, gk), g1 = __builtin_amdgcn_ds_bpermute(qb + 4, gk),
                      g2 = __builtin_amdgcn_ds_bpermute(qb + 8, gk), g3 = __builtin_amdgcn_ds_bpermute(qb + 12, gk);
        const int u = 4 * rt + (sc >> 2);
        if (ok && k == 0 && u < Ly.N) {
            const int32_t c_old = cg[u];
            const int32_t c_new = sat32(((int64_t)(int16_t)g0 * (int16_t)g1 + (int64_t)(int16_t)g2 * c_old) >> 15);
            const int16_t hv = sat16(((int32_t)tanh_q15(c_new, tt) * (int16_t)g3) >> 15);
            if (commit) cg[u] = c_new;
            out[u] = hv;
        }
        if (pk >= 0 && rb == rt0) DI_CLK_T(pk + 3, 0);
    }
}

// One workgroup per 16-stream tile, NN_WAVES_MAX waves at most: wave w runs
// row tiles w, w + waves, ... of every layer (an LSTM row tile holds whole
// units, so the waves' units and cell states are disjoint), wave 0 the
// context staging's share, the outputs and the post-processing.  A single
// stream (the drop-in NNSPClass_exec) runs its layers on eight waves: one
// wave walked every row tile's weight loads and MFMAs in sequence, ~30-75 us
// of the call's 54-97 us (rocprofv3, profiles/r05/dropin_nn/).
#define NN_WAVES_MAX 8
// DI (the drop-in kernel running out of LDS, NnRun.st_bytes > 0): the
// epilogue constants (ws, wsr, bs) and r's buffers point into LDS, and the
// layers from r.st_first on read their A fragments there too (Ast: NnImage.A's
// offsets rebased onto the LDS copy) -- the layer code inlined once per
// operand address space, so that each copy reads LDS or global memory directly
// (ALLST: every layer's fragments in LDS, the global copy not compiled -- its
// uniform values no longer crowd the scalar registers of the prologue)
template <bool DI, bool ALLST = false>
__device__ __forceinline__ void nn_body(const NnImage& img, NnRun r, const int32_t* ws, const int32_t* wsr,
                                        const int16_t* bs, const uint8_t* Ast, const int16_t* ttab = nullptr,
                                        int32_t* scr = nullptr) {
    __shared__ NnLds sm;
    // the activation table (DI: ttab, staged in LDS during the front end)
    const int16_t* const tt = DI ? ttab : sm.tanh_tbl;
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int nwv = (int)(blockDim.x >> 6);
    const bool w0 = wv == 0;
    const int sc = lane & 15;
    const int s0 = blockIdx.x * 16;
    const int s = s0 + sc;
    const bool valid = s < r.S;
    if (!DI)
        for (int i = threadIdx.x; i < 384; i += blockDim.x) sm.tanh_tbl[i] = nnsp_tbl_tanh[i];
    // LSTM state rows (neural_nets.c:27-42 layout: h int16[N], c int32[N]) of
    // stream gs, layer l: r.h / r.c + (gs * n_lstm + l) * hs
    const size_t hs = (size_t)r.hs;
    PostState ps = {};
    if (w0 && lane < 16 && valid && r.post) ps = reinterpret_cast<const PostState*>(r.post)[s];
    if (w0 && lane < 16) sm.slides[lane] = (valid && r.post) ? ps.slides : 1;
    __syncthreads();
    // (development probes of the prologue, nets of at most five layers: [7] its
    // first barrier passed, [8] the context staged, [9] the context barrier passed)
    if (DI && img.nl <= 5) DI_CLK(7);
    const int phase = r.mode == NN_MODE_DIRECT ? 0 : 1 - sm.slides[sc];
    // (DI: one frame, T == 1 checked at the launch -- the step loop known to
    // run once, so that nothing is hoisted out of it)
    const int T = DI || r.mode == NN_MODE_DIRECT ? 1 : r.T;
    const int nsteps = (T + 1) / 2;
    const int nl = r.nl_run;
    if (w0 && lane < 16 && valid && phase == 1 && r.trig) r.trig[(size_t)s * T] = ps.trigger;

    for (int j = 0; j < nsteps; ++j) {
        const int t = 2 * j + phase;
        const bool active = valid && t < T;
        if (w0 && lane < 16) sm.active[lane] = active;
        // ---- context window V[t..t+5], V = prev5 ++ feats (feature_module.c:54-57)
        {
            const int q = (int)(threadIdx.x >> 4) & 3, qs = 4 * nwv, q0 = q + 4 * wv;
            const int nch = r.mode == NN_MODE_DIRECT ? (img.L[0].K + 7) / 8 : 30;
            for (int cch = q0; cch < nch; cch += qs) {
                const int m = cch / 5, part = cch - 5 * m;
                int4 v = make_int4(0, 0, 0, 0);
                if (active) {
                    const int16_t* src;
                    if (!DI && r.mode == NN_MODE_DIRECT) {   // (DI: stream mode)
                        src = r.direct_in + (size_t)s * NN_MAX_K + 8 * cch;
                    } else {
                        const int idx = t + m;
                        src = idx < 5 ? r.prev5 + ((size_t)s * 5 + idx) * 40 + 8 * part
                                      : r.feats + ((size_t)s * r.T + (idx - 5)) * 40 + 8 * part;
                    }
                    v = *reinterpret_cast<const int4*>(src);
                }
                *reinterpret_cast<int4*>(&sm.act[0][sc][8 * cch]) = v;
            }
        }
        if (DI && img.nl <= 5 && j == 0) DI_CLK(8);
        __syncthreads();
        if (DI && img.nl <= 5 && j == 0) DI_CLK(9);
        int lst = 0;
        for (int i = 0; i < nl; ++i) {
            const NnLayer& Ly = img.L[i];
            const int16_t* in = &sm.act[i & 1][0][0];
            int16_t* out = &sm.act[(i + 1) & 1][0][0];
            if (Ly.type == NN_LSTM) {
                const int N = Ly.N;
                // the previous step's h stores (other lanes of this wave, below)
                // must be visible to these loads: an explicit workgroup-scope
                // fence rather than reliance on in-order vector memory
                __threadfence_block();
                for (int idx = threadIdx.x; idx < 16 * N; idx += blockDim.x) {   // stage h (the previous step's)
                    const int st = idx / N, u = idx - st * N, gs = s0 + st;
                    sm.h[st][u] = gs < r.S ? r.h[((size_t)gs * img.n_lstm + lst) * hs + u] : (int16_t)0;
                }
                __syncthreads();
                // (DI: every lane works for stream 0 -- its cell row and its activity)
                int32_t* cg = DI ? r.c + (size_t)lst * hs : (valid ? r.c + ((size_t)s * img.n_lstm + lst) * hs : nullptr);
                const bool commit = DI ? sm.active[0] != 0 : active;
                if (DI && (ALLST || i >= r.st_first))
                    lstm_layer_one(Ast, ws, wsr, bs, Ly, in, out, &sm.h[0][0], cg, tt, scr + 128 * wv, lane, commit,
                                   wv, nwv, NNSP_PROBES && r.probe && i < 8 ? 16 + 8 * i : -1);
                else if (DI)
                    lstm_layer_one(img.A, ws, wsr, bs, Ly, in, out, &sm.h[0][0], cg, tt, scr + 128 * wv, lane, commit,
                                   wv, nwv);
                else
                    lstm_layer_mfma(img.A, ws, wsr, bs, Ly, in, out, &sm.h[0][0], cg, tt, lane, commit, wv, nwv);
                __syncthreads();
                // h_state := output after all groups (lstm.c:205-206)
                for (int idx = threadIdx.x; idx < 16 * N; idx += blockDim.x) {
                    const int st = idx / N, u = idx - st * N, gs = s0 + st;
                    if (sm.active[st]) r.h[((size_t)gs * img.n_lstm + lst) * hs + u] = out[st * NN_ASTRIDE + u];
                }
                ++lst;
            } else {
                if (DI && (ALLST || i >= r.st_first))
                    fc_layer_mfma<DI>(Ast, ws, bs, Ly, in, out, tt, lane, wv, nwv,
                                  NNSP_PROBES && r.probe && i < 8 ? 16 + 8 * i : -1);
                else
                    fc_layer_mfma<DI>(img.A, ws, bs, Ly, in, out, tt, lane, wv, nwv);
            }
            if (NNSP_PROBES && r.probe && i < 8) DI_CLK_T(16 + 8 * i + 4, 0);
            __syncthreads();
            if (i < 8) DI_CLK(2 + i);   // (slots 10-13 taken)
        }
        const int16_t* fin = &sm.act[nl & 1][sc][0];
        const int nout = img.L[nl - 1].N;
        const bool lin = img.L[nl - 1].act == ACT_LINEAR;
        if (w0 && active && r.logits) {
            // each lane group q copies a quarter of its stream's outputs
            const int q = lane >> 4;
            if (r.mode == NN_MODE_DIRECT) {
                if (lin) {
                    int32_t* dst = reinterpret_cast<int32_t*>(r.logits) + (size_t)s * r.out_stride;
                    for (int o = q; o < nout; o += 4) dst[o] = reinterpret_cast<const int32_t*>(fin)[o];
                } else {
                    int16_t* dst = reinterpret_cast<int16_t*>(r.logits) + (size_t)s * r.out_stride * 2;
                    for (int o = q; o < nout; o += 4) dst[o] = fin[o];
                }
            } else {
                int32_t* dst = r.logits + ((size_t)s * T + t) * nout;
                for (int o = q; o < nout; o += 4)
                    dst[o] = lin ? reinterpret_cast<const int32_t*>(fin)[o] : (int32_t)fin[o];
            }
        }
        if (w0 && r.mode != NN_MODE_DIRECT && lane < 16 && active) {
            const LogitRow lg = {fin, lin};
            post_proc(ps, img, lg);
            if (r.trig) {
                r.trig[(size_t)s * T + t] = ps.trigger;
                if (t + 1 < T) r.trig[(size_t)s * T + t + 1] = ps.trigger;
            }
        }
        __syncthreads();
    }
    if (w0 && r.mode != NN_MODE_DIRECT && lane < 16 && valid && r.post) {
        ps.slides = (int16_t)(ps.slides ^ (T & 1));
        reinterpret_cast<PostState*>(r.post)[s] = ps;
    }
    DI_CLK(14);
    if (r.out_bytes) {   // the drop-in call's results, to mapped host memory (one workgroup)
        __threadfence();
        __syncthreads();
        for (int i = threadIdx.x; i < r.out_bytes / 16; i += blockDim.x)
            reinterpret_cast<int4*>(r.out_dst)[i] = reinterpret_cast<const int4*>(r.out_src)[i];
        DI_CLK(15);
#if NNSP_PROBES
        if (r.probe && threadIdx.x == 0) di_clk[11] = (long long)__builtin_amdgcn_s_memtime();
        if (r.probe && threadIdx.x == 0)
            for (int k = 0; k < NNSP_PROBE_LONGS; ++k) r.probe[k] = di_clk[k];
#endif
        if (r.done) {   // every wave's result stores complete at system scope, then the completion word
            __threadfence_system();
            __syncthreads();
            if (threadIdx.x == 0)
                __hip_atomic_store(r.done, (uint32_t)r.done_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}
__global__ __launch_bounds__(64 * NN_WAVES_MAX) void nn_kernel(NnImage img, NnRun r) {
    nn_body<false>(img, r, img.wsum, img.wsum_r, img.bias, nullptr);
}

// The drop-in call (NNSPClass_exec, one stream, one frame) in one launch: the
// front end (wave 0 has the frame), then the NN on eight waves; the barrier
// makes the front end's feature row visible to the NN's staging.
// ST (NnRun.st_bytes > 0): the call runs out of LDS.  The inputs are copied
// from mapped host memory into an LDS image of the staging buffer (in_dst's
// layout; every pointer into it rebased), and while wave 0 runs the frame the
// seven other waves copy the layers' epilogue constants and A fragments into
// LDS; the results go back to mapped host memory from the image.  Device
// memory is then read only for the tables and the weights that do not fit:
// each layer's memory round trips (fragments, constants, h / c, context) were
// most of its 1.4-4.6 us (dropin_kernel phase clocks, profiles/r06/).
// d[i] = s[i] for i = i0, i0 + NT, ... < n: U loads in flight per lane
template <int U, int NT>
__device__ __forceinline__ void lds_fill(int4* d, const int4* s, int n, int i0) {
    for (; i0 < n; i0 += NT * U) {
        int4 w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) w[u] = s[min(i0 + NT * u, n - 1)];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i0 + NT * u < n) d[i0 + NT * u] = w[u];
    }
}

// the drop-in call's inputs in the kernel arguments (KI): the launch writes
// them to device memory with the rest of the arguments, so that the kernel
// reads them from there instead of from mapped host memory across PCIe
template <bool KI>
struct DropinKin {
    int32_t unused;
};
template <>
struct DropinKin<true> {
    int4 b[NNSP_DROPIN_KARG_BYTES / 16];
};
// the waves without a frame (threadIdx.x >= 64): the epilogue constants, the
// activation table and the A fragments of layers st_first.. into the drop-in
// call's LDS (layout in di_call)
__device__ __forceinline__ void di_stage(const NnImage& img, const NnRun& r) {
    extern __shared__ __attribute__((aligned(16))) uint8_t di_lds[];
    const int ob = r.st_bytes, ow = ob + 4 * r.st_rows, oz = ow + 4 * r.st_rows, ot = oz + 2 * r.st_rows,
              osc = ot + 768, oa = osc + NN_WAVES_MAX * 512;
    {   // every line of the kernel arguments into the scalar cache (invalidated at
        // each launch), a few lines per wave, ahead of the NN's dependent reads
        typedef const uint32_t __attribute__((address_space(4))) * kptr;
        const kptr ka = (kptr)__builtin_amdgcn_kernarg_segment_ptr();
        constexpr int NL = (int)((sizeof(FeArgs) + sizeof(NnImage) + sizeof(NnRun) + 127) / 64);
        const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) - 1;
        uint32_t x = 0;
        for (int k = w; k < NL; k += NN_WAVES_MAX - 1) x ^= ka[16 * k];
        asm volatile("" ::"s"(x));
    }
    // every segment's first share in flight together (one round trip
    // for ~56 KB), the rest (nets wider than the reference's) after
    constexpr int NT = 64 * (NN_WAVES_MAX - 1), U = 16;
    const int t = (int)threadIdx.x - 64;
    const int nw = r.st_rows / 4, nz = r.st_rows / 8, na = r.st_abytes / 16;
    int4* dw = reinterpret_cast<int4*>(di_lds + ob);
    int4* dr = reinterpret_cast<int4*>(di_lds + ow);
    int4* dz = reinterpret_cast<int4*>(di_lds + oz);
    int4* da = reinterpret_cast<int4*>(di_lds + oa);
    const int4* sw = reinterpret_cast<const int4*>(img.wsum);
    const int4* sr = reinterpret_cast<const int4*>(img.wsum_r);
    const int4* sz = reinterpret_cast<const int4*>(img.bias);
    const int4* sa = reinterpret_cast<const int4*>(img.A + r.st_alo);
    // (clamped indexes: every load unconditional, into registers;
    // rows >= 16 and the image's A >= 1 KiB, so index 0 exists)
    const int4 cw = sw[min(t, nw - 1)], cr = sr[min(t, nw - 1)], cz = sz[min(t, nz - 1)];
    const int16_t ct = nnsp_tbl_tanh[min(t, 383)];
    int4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = sa[min(t + NT * u, max(na - 1, 0))];
    if (t < nw) {
        dw[t] = cw;
        dr[t] = cr;
    }
    if (t < nz) dz[t] = cz;
    if (t < 384) reinterpret_cast<int16_t*>(di_lds + ot)[t] = ct;
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (t + NT * u < na) da[t + NT * u] = v[u];
    lds_fill<U, NT>(dw, sw, nw, NT + t);
    lds_fill<U, NT>(dr, sr, nw, NT + t);
    lds_fill<U, NT>(dz, sz, nz, NT + t);
    lds_fill<U, NT>(da, sa, na, NT * U + t);
    if (NNSP_PROBES && r.probe) DI_CLK_T(12, 64);
}

// one drop-in call out of LDS (ST): dropin_kernel's body, and the resident
// worker's per request.  STAGE: the waves without a frame also stage the
// constants and A fragments (the worker stages them once, before its first
// request); seq: the completion word's value
template <bool PORT, bool KI, bool ALLST, bool STAGE>
__device__ __forceinline__ void di_call(const FeArgs& a, const NnImage& img, const NnRun& r, const DropinKin<KI>& kin,
                                        int32_t seq) {
    extern __shared__ __attribute__((aligned(16))) uint8_t di_lds[];
    // (r.st_base == a.in_dst: reading a's fields here as well made the
    // compiler keep a copy of FeArgs in scratch)
    const uint8_t* const dbase = reinterpret_cast<const uint8_t*>(r.st_base);
    // a pointer into the device staging buffer -> the same byte of the image
    auto rb = [&](const void* p) -> uint8_t* { return di_lds + (reinterpret_cast<const uint8_t*>(p) - dbase); };
    // LDS: image [0, st_bytes) | wsum | wsum_r [st_rows] int32 | bias [st_rows] int16 |
    // the activation table (384 int16) | the LSTM's per-wave scratch (2 x 64 int32) | A fragments
    const int ob = r.st_bytes, ow = ob + 4 * r.st_rows, oz = ow + 4 * r.st_rows, ot = oz + 2 * r.st_rows,
              osc = ot + 768, oa = osc + NN_WAVES_MAX * 512;
    if constexpr (KI)
        fe_body<FE_MODE_BATCH, PORT, 1, true>(a, di_lds, kin.b);
    else
        fe_body<FE_MODE_BATCH, PORT, 1, true>(a, di_lds);
    if (STAGE && threadIdx.x >= 64) di_stage(img, r);   // the waves without a frame: constants and fragments to LDS
    __syncthreads();
    DI_CLK(1);
    NnRun q = r;
    q.done_seq = seq;
    q.feats = reinterpret_cast<const int16_t*>(rb(r.feats));
    q.prev5 = reinterpret_cast<const int16_t*>(rb(r.prev5));
    q.h = reinterpret_cast<int16_t*>(rb(r.h));
    q.c = reinterpret_cast<int32_t*>(rb(r.c));
    q.post = rb(r.post);
    q.trig = reinterpret_cast<int16_t*>(rb(r.trig));
    q.out_src = rb(r.out_src);
    // (32-bit LDS addresses: NnImage.A offset st_alo lands on the copy's first byte)
    nn_body<true, ALLST>(img, q, reinterpret_cast<const int32_t*>(di_lds + ob), reinterpret_cast<const int32_t*>(di_lds + ow),
                  reinterpret_cast<const int16_t*>(di_lds + oz), di_lds + oa - r.st_alo,
                  reinterpret_cast<const int16_t*>(di_lds + ot), reinterpret_cast<int32_t*>(di_lds + osc));
}

template <bool PORT, bool ST, bool KI = false, bool ALLST = false>
__global__ __launch_bounds__(64 * NN_WAVES_MAX) void dropin_kernel(FeArgs a, NnImage img, NnRun r, DropinKin<KI> kin) {
#if NNSP_PROBES
    if (r.probe && threadIdx.x < NNSP_PROBE_LONGS) di_clk[threadIdx.x] = 0;   // (wave 0's own slots first)
#endif
    DI_CLK(0);
#if NNSP_PROBES
    if (r.probe && threadIdx.x == 0) di_clk[10] = (long long)__builtin_amdgcn_s_memtime();
#endif
    if constexpr (!ST) {
        fe_body<FE_MODE_BATCH, PORT, NN_WAVES_MAX, false, true>(a);
        __syncthreads();
        DI_CLK(1);
        nn_body<false>(img, r, img.wsum, img.wsum_r, img.bias, nullptr);
    } else {
        di_call<PORT, KI, ALLST, true>(a, img, r, kin, r.done_seq);
    }
}

// The resident drop-in worker (NNSP_DROPIN_WORKER): one workgroup that keeps a
// net's constants and A fragments in LDS and runs one call per request posted
// in mapped host memory, instead of one launch per call (the launch and the
// dispatch were ~10 us of every call).  mbox[0]: the request's sequence number,
// written by the host after the call's inputs are staged (seq0: the first
// request's); mbox[1]: stop.  Every wave leaves when stop is set or no request
// came for `idle` ticks of the 100 MHz clock, so the grid drains by itself.
// The arguments are those of every request it serves (the host compares them).
template <bool PORT, bool ALLST>
__global__ __launch_bounds__(64 * NN_WAVES_MAX) void dropin_worker_kernel(FeArgs a, NnImage img, NnRun r,
                                                                          const uint32_t* mbox, uint32_t seq0,
                                                                          long long idle) {
    __shared__ uint32_t wk_seq;
    const DropinKin<false> k0 = {0};
    uint32_t last = seq0 - 1u;
    if (threadIdx.x >= 64) di_stage(img, r);   // (wave 0 meanwhile waits for the first request)
    for (;;) {
        if (threadIdx.x == 0) {
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            uint32_t sq = last;
            for (;;) {   // (both words in one load: one trip across PCIe per poll)
                const unsigned long long v = __hip_atomic_load(reinterpret_cast<const unsigned long long*>(mbox),
                                                               __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                if ((uint32_t)v != last) {
                    sq = (uint32_t)v;
                    break;
                }
                if ((uint32_t)(v >> 32) != 0u) break;
                if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > idle) break;
                __builtin_amdgcn_s_sleep(1);
            }
            wk_seq = sq;
        }
        __syncthreads();
        const uint32_t sq = wk_seq;
        if (sq == last) break;   // stop, or idle: every wave leaves
        last = sq;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // (system scope: the staged inputs)
#if NNSP_PROBES
        if (r.probe && threadIdx.x < NNSP_PROBE_LONGS) di_clk[threadIdx.x] = 0;
#endif
        DI_CLK(0);
        di_call<PORT, false, ALLST, false>(a, img, r, k0, (int32_t)sq);
        __syncthreads();
    }
}

// prev5 := last 5 frames of V = prev5 ++ feats[b..T) after the segment; one
// block per stream, read all then write.
__global__ __launch_bounds__(64) void ctx_roll_kernel(int16_t* prev5, const int16_t* feats, int S, int T,
                                                     const int32_t* list, int n_list, const int32_t* seg_begin,
                                                     int seg_len) {
    const int i = blockIdx.x, c = threadIdx.x;   // c: 8-int16 chunk of the 5x40 context
    if (i >= (list ? n_list : S)) return;
    const int s = list ? list[i] : i;
    const int b = seg_begin ? seg_begin[s] : 0;
    const int L = (seg_len > 0 ? min(T, b + seg_len) : T) - b;
    if (L <= 0) return;
    int4 v = make_int4(0, 0, 0, 0);
    if (c < 25) {
        const int m = c / 5, part = c % 5, idx = L + m;
        v = idx < 5 ? *reinterpret_cast<const int4*>(prev5 + ((size_t)s * 5 + idx) * 40 + 8 * part)
                    : *reinterpret_cast<const int4*>(feats + ((size_t)s * T + b + idx - 5) * 40 + 8 * part);
    }
    __syncthreads();
    if (c < 25) *reinterpret_cast<int4*>(prev5 + (size_t)s * 200 + 8 * c) = v;
}

// tail := last 320 samples of (tail ++ input frames b..T-1), read all before writing.
__global__ __launch_bounds__(64) void tail_roll_kernel(int16_t* tail, const int16_t* pcm, int S, int T,
                                                      const int32_t* list, int n_list, const int32_t* seg_begin,
                                                      int seg_len, int lookback, const int16_t* hist, int H) {
    const int i = blockIdx.x;
    if (i >= (list ? n_list : S)) return;
    const int s = list ? list[i] : i;
    const int b = seg_begin ? seg_begin[s] : 0;
    const int L = (seg_len > 0 ? min(T, b + seg_len) : T) - b;
    if (L <= 0) return;
    int16_t v[5];
    for (int k = 0; k < 5; ++k) {
        const long long pos = 160LL * L + threadIdx.x + 64 * k;   // index into tail(320) ++ input(160 L)
        if (pos < 320) {
            v[k] = tail[(size_t)s * 320 + pos];
        } else {
            const long long n = pos - 320;
            const int x = b + (int)(n / 160) - lookback, o = (int)(n % 160);
            v[k] = x >= 0 ? pcm[((size_t)s * T + x) * 160 + o] : hist[((size_t)s * H + H + x) * 160 + o];
        }
    }
    __syncthreads();
    for (int k = 0; k < 5; ++k) tail[(size_t)s * 320 + threadIdx.x + 64 * k] = v[k];
}

// the common case of tail_roll (every stream, whole chunk, T >= 2, no
// look-back): the tail := the chunk's last two frames, 16 bytes per thread
__global__ __launch_bounds__(256) void tail_copy_kernel(uint4* tail, const int16_t* pcm, int S, int T) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;   // 40 uint4 per stream
    if (i >= 40LL * S) return;
    const int s = (int)(i / 40), c = (int)(i - 40LL * s);
    tail[i] = reinterpret_cast<const uint4*>(pcm + ((size_t)s * T + T - 2) * 160)[c];
}

// each net's normalised log-Mel of silence: mel 0 -> log10_vec's x == 0 -> 1
// (fixlog10.c:56), then feature_module.c:67-73
struct NringFill {
    int16_t* nring[3];
    const int32_t* nmean[3];
    const int32_t* nstdR[3];
    int32_t nshift[3];
};
__global__ __launch_bounds__(256) void nring_fill_kernel(NringFill f, int ring, const uint8_t* mask, int S) {
    const int s = blockIdx.x;
    if (s >= S || (mask && !mask[s])) return;
    const int32_t lg = log10_q15(0);
    for (int n = 0; n < 3; ++n) {
        if (!f.nring[n]) continue;
        for (int i = threadIdx.x; i < ring * 40; i += blockDim.x) {
            const int b = i % 40;
            f.nring[n][(size_t)s * ring * 40 + i] = sat16((((int64_t)lg - f.nmean[n][b]) * f.nstdR[n][b]) >> f.nshift[n]);
        }
    }
}

// ============================================================================
// Stage kernels (legacy scalar API + per-stage parity tests)
// ============================================================================
__global__ __launch_bounds__(64) void k_rfft(int32_t* x, int32_t* y, int n) {
    __shared__ __attribute__((aligned(16))) int32_t X[FE_X_DW + 272];   // + room for the padded T1
    __shared__ __attribute__((aligned(16))) FeTables TB;
    FeArgs none{};
    none.mode = FE_MODE_BATCH;
    fe_tables_init<false>(TB, none);
    const int lane = threadIdx.x;
    __syncthreads();
    for (int b = blockIdx.x; b < n; b += gridDim.x) {
        int32_t* xb = x + (size_t)b * 512;
        int32_t v[8];
        for (int m = 0; m < 4; ++m) {   // stage-1 layout: complex 64*m + lane
            v[2 * m] = xb[2 * (64 * m + lane)];
            v[2 * m + 1] = xb[2 * (64 * m + lane) + 1];
        }
        wave_cfft256<false>(v, X, TB, lane);
        int32_t* yb = y + (size_t)b * 1024;
        for (int m = 0; m < 4; ++m) {
            int32_t re, im;
            wave_split_bin<false>(X, TB, lane, m, re, im);
            const int k = lane + 64 * m;
            if (k) {
                yb[2 * k] = re; yb[2 * k + 1] = im;
                yb[1024 - 2 * k] = re; yb[1024 - 2 * k + 1] = wsub(0, im);
            }
        }
        if (lane == 0) {
            int32_t dc, nyq;
            wave_split_dc(X, dc, nyq);
            yb[0] = dc; yb[1] = 0; yb[512] = nyq; yb[513] = 0;
        }
        // pSrc holds the bit-reversed cFFT output afterwards (in-place CMSIS)
        for (int c = lane; c < 256; c += 64) {
            xb[2 * c] = X[2 * zslot(c)];
            xb[2 * c + 1] = X[2 * zslot(c) + 1];
        }
        wave_lds_sync();
    }
}

// The ARM_OPTIMIZED=0 build's rfft(512) (fft.c:27-126; cfft_only: its
// fft(8, ...), fft.c:128-221, natural-order output) on n vectors: x [n][512]
// (Frac15 reals, or 256 COMPLEX32), y [n][514] (bins 0..256) / [n][512].
// The input is not modified (rfft copies it into cinput, fft.c:53-57).
__global__ __launch_bounds__(64) void k_rfft_port(const int32_t* x, int32_t* y, int n, int cfft_only) {
    __shared__ __attribute__((aligned(16))) int32_t X[FE_X_DW + 272];   // + room for the padded T1
    __shared__ __attribute__((aligned(16))) FeTables TB;
    FeArgs none{};
    none.mode = FE_MODE_BATCH;
    fe_tables_init<true>(TB, none);
    const int lane = threadIdx.x;
    __syncthreads();
    for (int b = blockIdx.x; b < n; b += gridDim.x) {
        const int32_t* xb = x + (size_t)b * 512;
        int32_t v[8];
        for (int m = 0; m < 4; ++m) {   // stage-1 layout: complex 64*m + lane
            v[2 * m] = xb[2 * (64 * m + lane)];
            v[2 * m + 1] = xb[2 * (64 * m + lane) + 1];
        }
        wave_cfft256<true>(v, X, TB, lane);
        if (cfft_only) {
            int32_t* yb = y + (size_t)b * 512;
            for (int c = lane; c < 256; c += 64) {
                yb[2 * c] = X[2 * zslot(c)];
                yb[2 * c + 1] = X[2 * zslot(c) + 1];
            }
        } else {
            int32_t* yb = y + (size_t)b * 514;
            for (int m = 0; m < 4; ++m) {
                int32_t re, im;
                wave_split_bin<true>(X, TB, lane, m, re, im);
                const int k = lane + 64 * m;
                yb[2 * k] = re;
                yb[2 * k + 1] = im;
            }
            if (lane == 0) {
                const int2 z0 = *reinterpret_cast<const int2*>(X);
                yb[512] = wsub(wadd(z0.x, z0.x) >> 1, wadd(z0.y, z0.y) >> 1);
                yb[513] = 0;
            }
        }
        wave_lds_sync();
    }
}

// The ARM_OPTIMIZED=0 build's fft(exp_nfft, ...) and rfft(num_rfft, ...) for
// every size their tables serve (fft.c:27-221): exp_nfft 0..8 (radix-4 DIF
// stages for 8 and 7, then a radix-2 stage for 7; below that only the
// bit-reversal copy runs), rfft of 256 or 512 points.  One workgroup per call,
// butterflies across its 64 lanes, the working array in LDS.  Unlike the
// front end's register-resident 512-point path (k_rfft_port), this one keeps
// complex.c's int64 products and int32 clamps literally
// (complex32_interprod / _complex16_elmtprod), since for other inputs than
// windowed int16 PCM they can bind.
//   rfft: x = num_rfft int32 reals (not modified), y = num_rfft / 2 + 1 complex
//   fft:  x = 2^exp_nfft COMPLEX32, modified in place like fft.c's input; y =
//         2^exp_nfft COMPLEX32 in natural order
__device__ __forceinline__ int32_t clamp64(int64_t v) { return sat32(v); }
__device__ __forceinline__ int2 cmul_tw15(int2 a, int32_t w) {   // complex32_complex16_elmtprod, one element
    const int64_t wr = (int16_t)(w & 0xffff), wi = (int16_t)(w >> 16);
    return make_int2(clamp64(((int64_t)a.x * wr - (int64_t)a.y * wi) >> 15),
                     clamp64(((int64_t)a.x * wi + (int64_t)a.y * wr) >> 15));
}
__global__ __launch_bounds__(64) void k_fft_dif(int32_t* x, int32_t* y, int exp_nfft, int rfft) {
    __shared__ int2 c[256];
    __shared__ int2 z[256];
    const int lane = threadIdx.x;
    const int nfft = 1 << exp_nfft;
    for (int i = lane; i < nfft; i += 64) c[i] = make_int2(x[2 * i], x[2 * i + 1]);   // cinput (rfft: pairs of reals)
    __syncthreads();
    const int stages = exp_nfft == 8 ? 4 : (exp_nfft == 7 ? 3 : 0);
    int Nf = nfft, Ng = 1, S = 1 << (8 - exp_nfft);
    for (int st = 0; st < stages; ++st) {
        const int Nfd4 = Nf >> 2;
        for (int bf = lane; bf < Ng * Nfd4; bf += 64) {
            const int g = bf / Nfd4, m = bf - g * Nfd4, s0 = g * Nf + m, k = m * S;
            const int2 a = c[s0], b = c[s0 + 2 * Nfd4], cc = c[s0 + Nfd4], d = c[s0 + 3 * Nfd4];
            // ti = {x0, x2, x1, x3} (fft.c:180-187); to = M4 ti (exact sums, clamped, complex32_affine)
            const int64_t ar = a.x, ai = a.y, br = b.x, bi = b.y, cr = cc.x, ci = cc.y, dr = d.x, di = d.y;
            int2 to[4];
            to[0] = make_int2(clamp64(ar + br + cr + dr), clamp64(ai + bi + ci + di));
            to[1] = make_int2(clamp64(ar + br - cr - dr), clamp64(ai + bi - ci - di));
            to[2] = make_int2(clamp64(ar - br + ci - di), clamp64(ai - bi - cr + dr));   // row (1, -1, -j, j)
            to[3] = make_int2(clamp64(ar - br - ci + di), clamp64(ai - bi + cr - dr));   // row (1, -1, j, -j)
            for (int i = 0; i < 4; ++i) c[s0 + i * Nfd4] = cmul_tw15(to[i], nnsp_tbl_dif_tw[4 * k + i]);
        }
        __syncthreads();
        Nf >>= 2;
        Ng <<= 2;
        S <<= 2;
    }
    if (exp_nfft == 7) {   // the final radix-2 stage (fft.c:199-211): M2 = [[1, 1], [1, -1]]
        for (int m = lane; m < nfft / 2; m += 64) {
            const int2 p0 = c[2 * m], p1 = c[2 * m + 1];
            c[2 * m] = make_int2(clamp64((int64_t)p0.x + p1.x), clamp64((int64_t)p0.y + p1.y));
            c[2 * m + 1] = make_int2(clamp64((int64_t)p0.x - p1.x), clamp64((int64_t)p0.y - p1.y));
        }
        __syncthreads();
    }
    const int Rs = 8 - exp_nfft;
    for (int m = lane; m < nfft; m += 64) z[m] = c[nnsp_tbl_bitrev8[m] >> Rs];   // br_coeff[m] >> Rs
    __syncthreads();
    if (!rfft) {
        for (int m = lane; m < nfft; m += 64) {
            y[2 * m] = z[m].x;
            y[2 * m + 1] = z[m].y;
            x[2 * m] = c[m].x;   // fft() leaves its stage output in its input
            x[2 * m + 1] = c[m].y;
        }
        return;
    }
    // rfft's split (fft.c:62-125): Xe, Xo from Z and conj(Z(N/2 - i)), X = Xe + Xo tw^(R i)
    const int R = 1 << (8 - exp_nfft), half = nfft;   // num_rfft / 2 complex
    for (int i = lane; i < half; i += 64) {
        const int2 po = z[i], pr = z[i ? half - i : 0];
        const int32_t tr = pr.x, ti = wsub(0, pr.y);
        const int2 xe = make_int2(wadd(po.x, tr) >> 1, wadd(po.y, ti) >> 1);
        const int2 xo = make_int2(wsub(po.y, ti) >> 1, wsub(0, wsub(po.x, tr)) >> 1);
        const int2 o = cmul_tw15(xo, nnsp_tbl_dif_rtw[R * i]);
        y[2 * i] = wadd(xe.x, o.x);
        y[2 * i + 1] = wadd(xe.y, o.y);
        if (i == 0) {
            y[2 * half] = wsub(xe.x, xo.x);
            y[2 * half + 1] = wsub(xe.y, xo.y);
        }
    }
}

// complex.c's helpers (the drop-in complex.h), one launch per call: op codes
// NNSP_CPLX_* (nnsp_kabi.h); a, b: operands, o: result (b is written back by
// complex32_sub, which negates it in place, complex.c:108-113).  int64
// products with int32 clamps where complex.c has them, int32 wrap elsewhere.
__device__ __forceinline__ int64_t cx_re(int64_t ar, int64_t ai, int64_t br, int64_t bi) {
    return (int64_t)((uint64_t)(ar * br) - (uint64_t)(ai * bi));
}
__device__ __forceinline__ int64_t cx_im(int64_t ar, int64_t ai, int64_t br, int64_t bi) {
    return (int64_t)((uint64_t)(ar * bi) + (uint64_t)(ai * br));
}
__global__ __launch_bounds__(64) void k_cplx(int op, int32_t* o, int32_t* a, int32_t* b, int shift, int len, int32_t r,
                                             int32_t im) {
    const int n = op == NNSP_CPLX_INTERPROD || op == NNSP_CPLX_COPY || op == NNSP_CPLX_ADD || op == NNSP_CPLX_NEG ||
                          op == NNSP_CPLX_SUB || op == NNSP_CPLX_MUL || op == NNSP_CPLX_INIT
                      ? 1 : len;
    for (int i = threadIdx.x; i < n; i += 64) {
        switch (op) {
        case NNSP_CPLX_COPY:
        case NNSP_CPLX_INIT:         // o = a (complex32_init / real2cmplx: a staged by the host)
            o[0] = a[0];
            o[1] = a[1];
            break;
        case NNSP_CPLX_AFFINE:       // out[i] = interprod(input, Mat + i * len): a = Mat, b = input
        case NNSP_CPLX_INTERPROD: {  // out = sum a1[k] * a2[k]: a = arry1, b = arry2
            const int32_t* m = op == NNSP_CPLX_AFFINE ? a + 2 * (size_t)i * len : a;
            uint64_t re = 0, ii = 0;
            for (int k = 0; k < len; ++k) {
                re += (uint64_t)cx_re(b[2 * k], b[2 * k + 1], m[2 * k], m[2 * k + 1]);
                ii += (uint64_t)cx_im(b[2 * k], b[2 * k + 1], m[2 * k], m[2 * k + 1]);
            }
            o[2 * i] = sat32((int64_t)re >> shift);
            o[2 * i + 1] = sat32((int64_t)ii >> shift);
            break;
        }
        case NNSP_CPLX_ELMTPROD: {   // a: COMPLEX32, b: COMPLEX16 words
            const int64_t wr = (int16_t)(b[i] & 0xffff), wi = (int16_t)(b[i] >> 16);
            o[2 * i] = sat32(cx_re(a[2 * i], a[2 * i + 1], wr, wi) >> 15);
            o[2 * i + 1] = sat32(cx_im(a[2 * i], a[2 * i + 1], wr, wi) >> 15);
            break;
        }
        case NNSP_CPLX_ADD:
        case NNSP_CPLX_ARRY_ADD:
            o[2 * i] = wadd(a[2 * i], b[2 * i]);
            o[2 * i + 1] = wadd(a[2 * i + 1], b[2 * i + 1]);
            break;
        case NNSP_CPLX_NEG:
            o[0] = wsub(0, a[0]);
            o[1] = wsub(0, a[1]);
            break;
        case NNSP_CPLX_SUB: {        // neg(b, b); add(out, a, b)
            const int32_t nr = wsub(0, b[0]), ni = wsub(0, b[1]);
            b[0] = nr;
            b[1] = ni;
            o[0] = wadd(a[0], nr);
            o[1] = wadd(a[1], ni);
            break;
        }
        case NNSP_CPLX_MUL: {        // int32 products (complex.c:115-121), wrapping
            const uint32_t ar = a[0], ai = a[1], br = b[0], bi = b[1];
            o[0] = (int32_t)(ar * br - ai * bi);
            o[1] = (int32_t)(ar * bi + ai * br);
            break;
        }
        case NNSP_CPLX_ARRY_INIT:    // a: reals, b: imags (NULL: zeros, complexArry32_real2cmplx)
            o[2 * i] = a[i];
            o[2 * i + 1] = b ? b[i] : 0;
            break;
        }
    }
    (void)r;
    (void)im;
}

// spec2pspec_arm (shift 27) / spec2pspec (shift 15): x [n][1024], y [n][1024]
__global__ void k_pspec(int32_t* y, const int32_t* x, int len, int n, int shift) {
    const int b = blockIdx.y;
    if (b >= n) return;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < len; i += gridDim.x * blockDim.x) {
        const int32_t* xb = x + (size_t)b * 1024;
        y[(size_t)b * 1024 + i] = shift == 15 ? pspec15_of(xb[2 * i], xb[2 * i + 1]) : pspec_of(xb[2 * i], xb[2 * i + 1]);
    }
}

__global__ void k_mel(const int32_t* spec, int32_t* mel, int n) {
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int b = gid / 40, m = gid % 40;
    if (b >= n) return;
    int off = 0;
    for (int i = 0; i < m; ++i) off += 2 + nnsp_tbl_mel[off + 1] - nnsp_tbl_mel[off] + 1;
    const int st = nnsp_tbl_mel[off], en = nnsp_tbl_mel[off + 1];
    int64_t mac = 0;
    for (int j = st, o = off + 2; j <= en; ++j, ++o) mac += (int64_t)nnsp_tbl_mel[o] * spec[(size_t)b * 1024 + j];
    mel[(size_t)b * 40 + m] = sat32(mac >> 15);
}

__global__ void k_log10(int32_t* out, const int32_t* x, int n, int add) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = wadd(log10_q15(x[i]), add);
}

__global__ void k_act(int type, const int32_t* x, void* y, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (type == ACT_LINEAR)
        reinterpret_cast<int32_t*>(y)[i] = x[i];
    else
        reinterpret_cast<int16_t*>(y)[i] = type == ACT_RELU6 ? relu6_q12(x[i])
                                          : (type == ACT_TANH ? tanh_q15(x[i], nnsp_tbl_tanh)
                                                              : sigmoid_q15(x[i], nnsp_tbl_tanh));
}

// Scalar helpers of the legacy API: 0 ceiling, 1 compute_pwr2, 2 norm_oneTwo
// (out[2i] = y, out[2i+1] = shift), 3 my_argmax over n (out[0]).
__global__ void k_scalar(int op, const int32_t* in, int32_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (op == 3) {
        if (i == 0) out[0] = argmax_lw(in, n, 0);
        return;
    }
    if (i >= n) return;
    const int32_t x = in[i];
    if (op == 0) out[i] = ceiling_q15(x);
    else if (op == 1) out[i] = pwr2_q15(x);
    else {
        const uint32_t m = (uint32_t)x & 0x7FFFFFFFu;
        int sh = 0;
        if (m) sh = 15 - (31 - __clz((int)m));
        out[2 * i] = sh >= 0 ? wshl(x, sh) : (x >> -sh);
        out[2 * i + 1] = -sh;
    }
}

// binary_post_proc / s2i_post_proc on one stream's state; est is overwritten
// with the exp2 values for the binary case as the reference does (T7).
__global__ void k_post(int nn_id, int thresh_prob, int th_count, void* post, int32_t* est) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    PostState* ps = reinterpret_cast<PostState*>(post);
    NnImage im;
    im.nn_id = nn_id; im.thresh_prob = thresh_prob; im.th_count = th_count;
    int32_t lg[2] = {est[0], est[1]};
    if (nn_id == 0)
        post_proc(*ps, im, est);
    else
        post_proc(*ps, im, lg);
    if (nn_id != 0) {
        const int32_t mx = lg[0] > lg[1] ? lg[0] : lg[1];
        for (int i = 0; i < 2; ++i) est[i] = pwr2_q15(sat32(((int64_t)wsub(lg[i], mx) * 0xB8AA) >> 15));
    }
}

// FeatureClass_setDefault (feature_module.c:26-45) for n streams: ctx slots 0-4.
__global__ void k_fe_default(int16_t* prev5, int16_t* tail, const int32_t* mean, const int32_t* stdR,
                             int norm_shift, const uint8_t* mask, int n) {
    const int gid = blockIdx.x * blockDim.x + threadIdx.x;
    const int s = gid / 40, m = gid % 40;
    if (s >= n || (mask && !mask[s])) return;
    int64_t v = (int64_t)wsub(-147963, mean[m]);
    const int16_t q = sat16((v * stdR[m]) >> norm_shift);
    // after reset ctx = [q q q q q X]; the next frame sees V[0..4] = [q q q q X]
    const int16_t X = prev5[((size_t)s * 5 + 4) * 40 + m];
    for (int j = 0; j < 4; ++j) prev5[((size_t)s * 5 + j) * 40 + m] = q;
    prev5[((size_t)s * 5 + 4) * 40 + m] = X;
    for (int i = m; i < 320; i += 40) tail[(size_t)s * 320 + i] = 0;
}

// NNSPClass_reset post/NN part (nn_speech.c:57-72, neural_nets.c:27-42)
// (row: h / c elements per stream, n_lstm * hs)
__global__ void k_nn_default(int16_t* h, int32_t* c, void* post, int row, const uint8_t* mask, int n) {
    const int s = blockIdx.x;
    if (s >= n || (mask && !mask[s])) return;
    for (int i = threadIdx.x; i < row; i += blockDim.x) {
        h[(size_t)s * row + i] = 0;
        c[(size_t)s * row + i] = 0;
    }
    if (threadIdx.x == 0 && post) {
        PostState* p = reinterpret_cast<PostState*>(post) + s;
        p->slides = 1;
        p->trigger = 0;
        for (int i = 0; i < 7; ++i) p->counts[i] = 0;
        p->outputs[0] = p->outputs[1] = p->outputs[2] = 0;
        p->argmax_last = 0;
    }
}

// Legacy row-block primitives (RowArgs, nnsp_kabi.h): one thread per output
// row of a layer stored as 4-row groups, remainder group last (fc_8x16 /
// rc_8x16, affine.c:409-563).  Byte of (row r, column c of a pair) inside a
// group's column pair of R rows (Appendix B of SURVEY; affine.c:80-149):
__device__ __forceinline__ int rows_wofs(int R, int r, int c) {
    return R == 4 ? (r >> 1) * 4 + 2 * c + (r & 1) : (R == 3 ? (r < 2 ? 2 * c + r : 4 + c) : (R == 2 ? 2 * c + r : c));
}
// sum_k W[i][k] x[k] of row i (the SMLALD pairs, then the odd-column tail)
// port: the ARM_OPTIMIZED=0 order (affine.c:261-346), per column pair, per row
__device__ int64_t rows_dot(const int8_t* w, const int16_t* x, int K, int rows, int i, int port) {
    const int g = i >> 2, r = i & 3, R = min(4, rows - 4 * g);
    const int8_t* wg = w + (size_t)g * 4 * K;
    const int o0 = port ? 2 * r : rows_wofs(R, r, 0), o1 = port ? 2 * r + 1 : rows_wofs(R, r, 1);
    int64_t s = 0;
    for (int p = 0; p < (K >> 1); ++p)
        s += (int64_t)wg[2 * R * p + o0] * x[2 * p] + (int64_t)wg[2 * R * p + o1] * x[2 * p + 1];
    if (K & 1) s += (int64_t)wg[(K >> 1) * 2 * R + r] * x[K - 1];
    return s;
}
__device__ __forceinline__ int64_t wrap32(int64_t v) { return (int64_t)(int32_t)(uint32_t)(uint64_t)v; }

// affine_Krows_8x16 (affine.c:12-259; _acc32b affine_acc32b.c:12-260) and
// rc_Krows_8x16 (affine.c:348-407): accumulate, (rc: shift by qir - qi and add
// the recurrent half), bias aligned to qbit_s, then if is_out the output
// shift, clamp (acc64) and activation.  The "align acc" shift_64b on
// pt_accum (affine.c:186-187) acts on values the sums then overwrite (T1).
__global__ void k_rows(RowArgs a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.rows) return;
    int64_t s;
    int qs;
    if (a.mode == ROWS_RC) {
        int64_t s1 = rows_dot(a.w, a.x, a.K, a.rows, i, a.port);   // no bias: qbit_s = qi + qk
        if (a.acc32) s1 = shift32((int32_t)wrap32(s1), a.qir - a.qi);
        else s1 = shift64(s1, a.qir - a.qi);
        s = s1 + rows_dot(a.wr, a.xr, a.Kr, a.rows, i, a.port);
        qs = a.b ? max(15, a.qir + a.qk) : a.qir + a.qk;
    } else {
        s = a.acc[i] + rows_dot(a.w, a.x, a.K, a.rows, i, a.port);
        qs = a.b ? max(15, a.qi + a.qk) : a.qi + a.qk;
    }
    if (a.acc32) s = wrap32(s);
    if (a.port) {   // the ARM_OPTIMIZED=0 build's live align shift (affine.c:311-313): 0 without a bias
        const int al = qs - (a.mode == ROWS_RC ? a.qir : a.qi) - a.qk;
        s = a.acc32 ? (int64_t)shift32((int32_t)s, al) : shift64(s, al);
    }
    if (a.b) {
        const int sh = qs - a.qb;
        const int16_t bv = a.b[i];
        if (a.acc32)
            s = wadd((int32_t)s, sh >= 0 ? wshl(bv, sh) : ((int32_t)bv >> -sh));
        else
            s += sh >= 0 ? (int64_t)((uint64_t)(int64_t)bv << sh) : ((int64_t)bv >> -sh);
    }
    // is_out: shift_64b/32b(pt_accum, 15 - qbit_s) in place, then clamp (acc64) and act (affine.c:242-253)
    if (a.is_out) s = a.acc32 ? (int64_t)shift32((int32_t)s, 15 - qs) : shift64(s, 15 - qs);
    if (a.mode == ROWS_AFFINE) a.acc[i] = s;
    if (a.is_out && a.out) {
        const int32_t v = a.acc32 ? (int32_t)s : sat32(s);
        if (a.act == ACT_LINEAR)
            reinterpret_cast<int32_t*>(a.out)[i] = v;
        else
            reinterpret_cast<int16_t*>(a.out)[i] = a.act == ACT_RELU6 ? relu6_q12(v)
                                                 : (a.act == ACT_TANH ? tanh_q15(v, nnsp_tbl_tanh)
                                                                      : sigmoid_q15(v, nnsp_tbl_tanh));
    }
}

__global__ void k_shift(void* x, int sh, int n, int acc32) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (acc32) {
        int32_t* p = reinterpret_cast<int32_t*>(x);
        p[i] = shift32(p[i], sh);
    } else {
        int64_t* p = reinterpret_cast<int64_t*>(x);
        p[i] = shift64(p[i], sh);
    }
}

// Synthetic PCM (bench / tests): SplitMix64(seed, stream, sample) -> int16 in
// [-amp, amp-1]; identical to oracle.synthetic_pcm.  With wavs:
// every `every`-th stream g (g % every == 0) instead replays wav
// (g / every) % n_wavs cyclically from sample offset (g * 1601) mod wav_len.
__global__ void k_synth_pcm(int16_t* out, int S, int T, unsigned long long seed, int s0, long long t0, int amp,
                            const int16_t* wavs, int n_wavs, int wav_len, int every) {
    const long long n = (long long)S * T * 160;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        const unsigned long long s = (unsigned long long)(i / (160LL * T)) + (unsigned long long)s0;
        const unsigned long long k = (unsigned long long)(i % (160LL * T)) + (unsigned long long)t0 * 160ULL;
        if (wavs && every > 0 && s % (unsigned long long)every == 0) {
            const unsigned long long w = (s / (unsigned long long)every) % (unsigned long long)n_wavs;
            const unsigned long long L = (unsigned long long)wav_len;
            out[i] = wavs[w * L + (s * 1601ULL % L + k) % L];
            continue;
        }
        unsigned long long z = seed + s * 0x9E3779B97F4A7C15ULL + k * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        z = z ^ (z >> 31);
        out[i] = (int16_t)((long long)(z % (unsigned long long)(2 * amp)) - amp);
    }
}

// the front end's per-workgroup tables into a global image (nnspk_build_fe_tables)
template <bool PORT>
__global__ __launch_bounds__(256) void fe_tables_build_kernel(FeTables* out, FeArgs a) {
    fe_tables_init<PORT>(*out, a);
    if (threadIdx.x < 64) {
        FeLane L;
        fe_lane_init(L, threadIdx.x);
        FeLaneImg* li = reinterpret_cast<FeLaneImg*>(out + 1);
        li->mj0[threadIdx.x] = L.mj0;
        li->mfirst[threadIdx.x] = L.mfirst;
        li->mcnt[threadIdx.x] = L.mcnt;
    }
}

// ============================================================================
// C-ABI launch layer (plain pointers; stream passed as void*)
// ============================================================================
static int ok(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }

extern "C" {

int nnspk_build_fe_tables(void** out, const FeArgs* a, void* stream) {
    *out = nullptr;
    FeTables* t = nullptr;
    hipError_t e = hipMalloc((void**)&t, sizeof(FeTables) + sizeof(FeLaneImg));
    if (e != hipSuccess) return (int)e;
    if (a->port)
        hipLaunchKernelGGL(fe_tables_build_kernel<true>, dim3(1), dim3(256), 0, (hipStream_t)stream, t, *a);
    else
        hipLaunchKernelGGL(fe_tables_build_kernel<false>, dim3(1), dim3(256), 0, (hipStream_t)stream, t, *a);
    e = hipGetLastError();
    if (e != hipSuccess) {
        (void)hipFree(t);
        return (int)e;
    }
    *out = t;
    return 0;
}

int nnspk_launch_fe(const FeArgs* a, void* stream) {
    const int nrow = a->n_list_dev ? a->S : (a->list ? a->n_list : a->S);
    if (nrow <= 0 || a->T <= 0) return 0;
    int W = a->seg_len > 0 && a->seg_len < a->T ? a->seg_len : a->T;
    if (a->mode == FE_MODE_COLD && W > 2) W = 2;
    const long long nfr = (long long)nrow * W;
    // seven-wave workgroups for the shared mode of the shipped build (FeGeom)
    const bool seven = a->mode == FE_MODE_SHARED && !a->port && FeGeom<FE_MODE_SHARED, false>::seven;
    const int wpg = seven ? FeGeom<FE_MODE_SHARED, false>::WPG : FE_WPG;
    const int per_cu = seven ? FeGeom<FE_MODE_SHARED, false>::PER_CU : 24 / FE_WPG;
    long long blocks = (nfr + wpg - 1) / wpg;
    // whole multiples of the resident workgroups (256 CUs x 6 at 80 VGPRs):
    // each wave runs a contiguous frame range, so a partial last wave of
    // workgroups is pure tail
    // (grid sweep, profiles/fe_sweep.sh: 3072 -> 454 M, 6144 -> 460 M cascade frames/s)
    // (also measured in round 3, paired A/B: 1536 blocks -- one generation --
    // 882 M, 3072 951 M, 6144 965 M, 12288 965 M, 24576 954 M cascade frames/s:
    // the later generations' workgroup turnover lets the nets' rounds in)
    // (round 3, with the prebuilt tables -- staging 22 -> 10.6 us per
    // workgroup -- eight generations, 67 frames per wave: cascade 3 072
    // workgroups 0.948 G, 4 608 0.980, 6 144 0.986-0.998, 9 216 0.992,
    // 12 288 1.016, 18 432 1.008, 24 576 0.992 G; shared FE 2.16 -> 2.09 ms)
    // (round 4, the final front end -- 72 VGPRs, ~307 VALU per frame -- paired
    // A/B over two sweeps, profiles/r04/fe_gens/: shared FE 1.99 ms at eight
    // generations, 1.95 at six, 1.96 at ten and twelve; cascade 1.171 / 1.183 /
    // 1.178 / 1.179 G: six generations, 9 216 workgroups, since then)
    // (NNSP_FE_GENS, development: another number of generations)
    static const long long gens = [] {
        const char* e = getenv("NNSP_FE_GENS");
        return e && atoll(e) > 0 ? atoll(e) : 6LL;
    }();
    const long long cap = 256LL * per_cu * gens;
    if (blocks > cap) blocks = cap;
    // cold frames (<= 2 per reset, device-sized list): enough workgroups for
    // about one frame per wave -- their latency sits on each round's critical path
    if (a->mode == FE_MODE_COLD && a->n_list_dev) {
        // (NNSP_COLD_FE_BLOCKS, development: another cap for the device-sized lists)
        static const long long cold_cap = [] {
            const char* e = getenv("NNSP_COLD_FE_BLOCKS");
            return e && atoll(e) > 0 ? atoll(e) : 8192LL / FE_WPG;
        }();
        if (blocks > cold_cap) blocks = cold_cap;
    }
    const dim3 g((unsigned)blocks), blk(64 * wpg);
    hipStream_t st = (hipStream_t)stream;
    // two frames per wave (fe_kernel2): FE_PAIR_DEFAULT = 0 off, 1 the batch
    // mode only (default), 2 the shared mode too.  Measured (A/B on one box):
    // batch FE 0.55 -> 0.52 ms (VAD, 8192 streams); shared FE 2.18 -> 2.34 ms
    // (fewer waves per SIMD keep its VALU less busy: SQ_ACTIVE_INST_VALU 95 -> 88 %)
    constexpr int pair = FE_PAIR_DEFAULT;
    const bool use_pair = a->mode == FE_MODE_BATCH ? pair >= 1 : (a->mode == FE_MODE_SHARED && pair >= 2);
    // (no segments: every frame of a listed row is inside the chunk)
    if (use_pair && !a->seg_begin && !a->dbg_spec && !a->dbg_log && !a->dbg_clk) {
        // whole multiples of the resident workgroups at four per CU
        long long b2 = (nfr + 7) / 8;
        // (round 3, prebuilt tables: 4 096 workgroups 1.196 G VAD frames/s,
        // 6 144 1.169, 8 192 1.192, 12 288 1.156 -- four generations stay)
        if (b2 > 256LL * 4 * 4) b2 = 256LL * 4 * 4;
        const dim3 g2((unsigned)b2), blk2(256);
        if (a->mode == FE_MODE_SHARED) {
            if (a->port) hipLaunchKernelGGL((fe_kernel2<FE_MODE_SHARED, true>), g2, blk2, 0, st, *a);
            else hipLaunchKernelGGL((fe_kernel2<FE_MODE_SHARED, false>), g2, blk2, 0, st, *a);
        } else {
            if (a->port) hipLaunchKernelGGL((fe_kernel2<FE_MODE_BATCH, true>), g2, blk2, 0, st, *a);
            else hipLaunchKernelGGL((fe_kernel2<FE_MODE_BATCH, false>), g2, blk2, 0, st, *a);
        }
        return ok(hipGetLastError());
    }
    if (a->mode == FE_MODE_SHARED) {
        if (a->port) hipLaunchKernelGGL((fe_kernel<FE_MODE_SHARED, true>), g, blk, 0, st, *a);
        else hipLaunchKernelGGL((fe_kernel<FE_MODE_SHARED, false>), g, blk, 0, st, *a);
    } else if (a->mode == FE_MODE_COLD) {
        if (a->port) hipLaunchKernelGGL((fe_kernel<FE_MODE_COLD, true>), g, blk, 0, st, *a);
        else hipLaunchKernelGGL((fe_kernel<FE_MODE_COLD, false>), g, blk, 0, st, *a);
    } else {
        if (a->port) hipLaunchKernelGGL((fe_kernel<FE_MODE_BATCH, true>), g, blk, 0, st, *a);
        else hipLaunchKernelGGL((fe_kernel<FE_MODE_BATCH, false>), g, blk, 0, st, *a);
    }
    return ok(hipGetLastError());
}

int nnspk_launch_rows(const RowArgs* a, void* stream) {
    if (a->rows <= 0) return 0;
    hipLaunchKernelGGL(k_rows, dim3((a->rows + 63) / 64), dim3(64), 0, (hipStream_t)stream, *a);
    return ok(hipGetLastError());
}

int nnspk_launch_shift(void* x, int shift, int n, int acc32, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_shift, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, x, shift, n, acc32);
    return ok(hipGetLastError());
}

int nnspk_launch_nring_fill(int16_t* const nring[3], const int32_t* const nmean[3], const int32_t* const nstdR[3],
                            const int32_t nshift[3], int ring, const uint8_t* mask, int S, void* stream) {
    if (S <= 0) return 0;
    NringFill f;
    for (int n = 0; n < 3; ++n) {
        f.nring[n] = nring[n];
        f.nmean[n] = nmean[n];
        f.nstdR[n] = nstdR[n];
        f.nshift[n] = nshift[n];
    }
    hipLaunchKernelGGL(nring_fill_kernel, dim3(S), dim3(256), 0, (hipStream_t)stream, f, ring, mask, S);
    return ok(hipGetLastError());
}

// the drop-in call's LDS layout (ST): rows of epilogue constants, the bytes
// before the A fragments, and the smallest first layer whose fragments through
// the last layer's fit beside lds_static; 1: the image and the constants do
// not fit (the device-memory kernel runs the call)
static int di_rows(const NnImage* img) {
    int rows = 0;
    for (int i = 0; i < img->nl; ++i) {
        const int e = img->L[i].ep_off + 16 * img->L[i].nrt;
        rows = e > rows ? e : rows;
    }
    return rows;   // (multiples of 16)
}
static size_t di_fixed(const NnImage* img, const NnRun* r) {   // + the tanh table, the LSTM scratch
    return (size_t)(r->st_bytes > 0 ? r->st_bytes : 0) + 10 * (size_t)di_rows(img) + 768 + NN_WAVES_MAX * 512;
}
static bool di_fits(const NnImage* img, const NnRun* r) {   // (the LDS kernels' static LDS is < 56 KB)
    return r->st_bytes > 0 && di_fixed(img, r) <= 160 * 1024 - 56 * 1024;
}
static int di_layout(const FeArgs* a, const NnImage* img, const NnRun* r, size_t lds_static, NnRun* rr, size_t* dyn) {
    if (!a->in_dst || !a->in_bytes || !r->out_bytes || (r->st_bytes & 15) || a->in_bytes > r->st_bytes)
        return ok(hipErrorInvalidValue);
    const size_t fixed = di_fixed(img, r), cap = 160 * 1024 - lds_static;
    if (fixed > cap) return ok(hipErrorInvalidValue);   // (checked against a bound before)
    int first = r->nl_run;
    int64_t lo = 0, hi = 0;
    for (int f = r->nl_run - 1; f >= 0; --f) {
        int64_t l = INT64_MAX, h = 0;
        for (int i = f; i < r->nl_run; ++i) {
            const NnLayer& L = img->L[i];
            const int64_t e = L.a_off + (int64_t)L.nrt * L.nkt * 1024;
            l = L.a_off < l ? L.a_off : l;
            h = e > h ? e : h;
            if (L.type == NN_LSTM) {
                const int64_t er = L.ar_off + (int64_t)L.nrt * L.nkt_r * 1024;
                l = L.ar_off < l ? L.ar_off : l;
                h = er > h ? er : h;
            }
        }
        if (fixed + (size_t)(h - l) > cap) break;
        first = f;
        lo = l;
        hi = h;
    }
    *rr = *r;
    rr->st_base = a->in_dst;
    rr->st_rows = di_rows(img);
    rr->st_first = first;
    rr->st_alo = lo;
    rr->st_abytes = (int32_t)(hi - lo);   // (a_off: multiples of 1 KiB)
    *dyn = fixed + (size_t)(hi - lo);
    return 0;
}
// a kernel's static LDS, and its dynamic LDS limit raised to the rest (once per kernel)
static int di_prepare(const void* fn, size_t* lds_static) {
    if (*lds_static) return 0;
    hipFuncAttributes fa;
    hipError_t e = hipFuncGetAttributes(&fa, fn);
    if (e != hipSuccess) return ok(e);
    e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - (int)fa.sharedSizeBytes);
    if (e != hipSuccess) return ok(e);
    *lds_static = fa.sharedSizeBytes;
    return 0;
}

int nnspk_launch_dropin(const FeArgs* a, const NnImage* img, const NnRun* r, const void* kin, void* stream) {
    if (a->S != 1 || a->T != 1 || a->mode != FE_MODE_BATCH || r->S != 1 || r->T != 1) return ok(hipErrorInvalidValue);
    if (img->n_lstm && r->hs < 8) return ok(hipErrorInvalidValue);
    const DropinKin<false> k0 = {0};
    // out of LDS when the image and every layer's constants fit beside the
    // kernel's static LDS (a net of very many rows runs from device memory)
    if (!di_fits(img, r)) {
        if (a->port)
            hipLaunchKernelGGL((dropin_kernel<true, false>), dim3(1), dim3(64 * NN_WAVES_MAX), 0, (hipStream_t)stream, *a, *img, *r, k0);
        else
            hipLaunchKernelGGL((dropin_kernel<false, false>), dim3(1), dim3(64 * NN_WAVES_MAX), 0, (hipStream_t)stream, *a, *img, *r, k0);
        return ok(hipGetLastError());
    }
    // out of LDS: the image, the constants, and the A fragments of as many
    // trailing layers as fit beside the kernel's static LDS.  The variants:
    // port + 2 KI (the inputs in the kernel arguments when they fit) + 4 ALLST
    // (every layer's fragments in LDS); one static LDS size
    static const void* const fns[8] = {
        reinterpret_cast<const void*>(dropin_kernel<false, true, false, false>),
        reinterpret_cast<const void*>(dropin_kernel<true, true, false, false>),
        reinterpret_cast<const void*>(dropin_kernel<false, true, true, false>),
        reinterpret_cast<const void*>(dropin_kernel<true, true, true, false>),
        reinterpret_cast<const void*>(dropin_kernel<false, true, false, true>),
        reinterpret_cast<const void*>(dropin_kernel<true, true, false, true>),
        reinterpret_cast<const void*>(dropin_kernel<false, true, true, true>),
        reinterpret_cast<const void*>(dropin_kernel<true, true, true, true>)};
    static size_t lds_static[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int e = di_prepare(fns[0], &lds_static[0]);
    if (e) return e;
    NnRun rr;
    size_t dyn = 0;
    e = di_layout(a, img, r, lds_static[0], &rr, &dyn);
    if (e) return e;
    const int ki = kin && a->in_bytes <= NNSP_DROPIN_KARG_BYTES;
    const int fx = (a->port ? 1 : 0) + (ki ? 2 : 0) + (rr.st_first == 0 ? 4 : 0);
    e = di_prepare(fns[fx], &lds_static[fx]);
    if (e) return e;
    if (lds_static[fx] != lds_static[0]) return ok(hipErrorInvalidValue);
#define NNSP_DI_LAUNCH(P, K, AL, KARG)                                                                              \
    hipLaunchKernelGGL((dropin_kernel<P, true, K, AL>), dim3(1), dim3(64 * NN_WAVES_MAX), dyn, (hipStream_t)stream, \
                       *a, *img, rr, KARG)
    if (ki) {
        DropinKin<true> k;
        memcpy(k.b, kin, (size_t)a->in_bytes);
        switch (fx) {
        case 2: NNSP_DI_LAUNCH(false, true, false, k); break;
        case 3: NNSP_DI_LAUNCH(true, true, false, k); break;
        case 6: NNSP_DI_LAUNCH(false, true, true, k); break;
        default: NNSP_DI_LAUNCH(true, true, true, k); break;
        }
    } else {
        switch (fx) {
        case 0: NNSP_DI_LAUNCH(false, false, false, k0); break;
        case 1: NNSP_DI_LAUNCH(true, false, false, k0); break;
        case 4: NNSP_DI_LAUNCH(false, false, true, k0); break;
        default: NNSP_DI_LAUNCH(true, false, true, k0); break;
        }
    }
#undef NNSP_DI_LAUNCH
    return ok(hipGetLastError());
}

int nnspk_dropin_worker_ok(const NnImage* img, const NnRun* r) { return di_fits(img, r) ? 1 : 0; }

int nnspk_launch_dropin_worker(const FeArgs* a, const NnImage* img, const NnRun* r, const uint32_t* mbox,
                               uint32_t seq0, long long idle_ticks, void* stream) {
    if (a->S != 1 || a->T != 1 || a->mode != FE_MODE_BATCH || r->S != 1 || r->T != 1 || !mbox || idle_ticks <= 0)
        return ok(hipErrorInvalidValue);
    if ((img->n_lstm && r->hs < 8) || !di_fits(img, r) || !r->done) return ok(hipErrorInvalidValue);
    static const void* const fns[4] = {reinterpret_cast<const void*>(dropin_worker_kernel<false, false>),
                                       reinterpret_cast<const void*>(dropin_worker_kernel<true, false>),
                                       reinterpret_cast<const void*>(dropin_worker_kernel<false, true>),
                                       reinterpret_cast<const void*>(dropin_worker_kernel<true, true>)};
    static size_t lds_static[4] = {0, 0, 0, 0};
    int e = di_prepare(fns[0], &lds_static[0]);
    if (e) return e;
    NnRun rr;
    size_t dyn = 0;
    e = di_layout(a, img, r, lds_static[0], &rr, &dyn);
    if (e) return e;
    const int fx = (a->port ? 1 : 0) + (rr.st_first == 0 ? 2 : 0);
    e = di_prepare(fns[fx], &lds_static[fx]);
    if (e) return e;
    if (lds_static[fx] != lds_static[0]) return ok(hipErrorInvalidValue);
    const dim3 g(1), b(64 * NN_WAVES_MAX);
    const hipStream_t s = (hipStream_t)stream;
    switch (fx) {
    case 0: hipLaunchKernelGGL((dropin_worker_kernel<false, false>), g, b, dyn, s, *a, *img, rr, mbox, seq0, idle_ticks); break;
    case 1: hipLaunchKernelGGL((dropin_worker_kernel<true, false>), g, b, dyn, s, *a, *img, rr, mbox, seq0, idle_ticks); break;
    case 2: hipLaunchKernelGGL((dropin_worker_kernel<false, true>), g, b, dyn, s, *a, *img, rr, mbox, seq0, idle_ticks); break;
    default: hipLaunchKernelGGL((dropin_worker_kernel<true, true>), g, b, dyn, s, *a, *img, rr, mbox, seq0, idle_ticks); break;
    }
    return ok(hipGetLastError());
}

int nnspk_launch_nn(const NnImage* img, const NnRun* r, void* stream) {
    if (r->S <= 0) return 0;
    if (img->n_lstm && r->hs < 8) return ok(hipErrorInvalidValue);   // h / c row stride unset
    // few tiles (the drop-in single stream): eight waves per tile share each
    // layer's row tiles; many: one wave per tile, many tiles per CU
    const int tiles = (r->S + 15) / 16;
    const int waves = tiles <= 32 ? NN_WAVES_MAX : 1;
    hipLaunchKernelGGL(nn_kernel, dim3(tiles), dim3(64 * waves), 0, (hipStream_t)stream, *img, *r);
    return ok(hipGetLastError());
}

int nnspk_launch_ctx_roll(int16_t* prev5, const int16_t* feats, int S, int T, const int32_t* list, int n_list,
                          const int32_t* seg_begin, int seg_len, void* stream) {
    const int n = list ? n_list : S;
    if (n <= 0) return 0;
    hipLaunchKernelGGL(ctx_roll_kernel, dim3(n), dim3(64), 0, (hipStream_t)stream, prev5, feats, S, T, list, n_list,
                       seg_begin, seg_len);
    return ok(hipGetLastError());
}

int nnspk_launch_tail_roll(int16_t* tail, const int16_t* pcm, int S, int T, const int32_t* list, int n_list,
                           const int32_t* seg_begin, int seg_len, int lookback, const int16_t* hist,
                           int hist_frames, void* stream) {
    const int n = list ? n_list : S;
    if (n <= 0) return 0;
    if (!list && !seg_begin && (seg_len <= 0 || seg_len >= T) && lookback == 0 && T >= 2 && ((uintptr_t)pcm & 15) == 0 && ((uintptr_t)tail & 15) == 0) {
        const long long nv = 40LL * S;
        hipLaunchKernelGGL(tail_copy_kernel, dim3((unsigned)((nv + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                           reinterpret_cast<uint4*>(tail), pcm, S, T);
        return ok(hipGetLastError());
    }
    hipLaunchKernelGGL(tail_roll_kernel, dim3(n), dim3(64), 0, (hipStream_t)stream, tail, pcm, S, T, list, n_list,
                       seg_begin, seg_len, lookback, hist, hist_frames);
    return ok(hipGetLastError());
}

int nnspk_launch_synth_pcm(int16_t* out, int S, int T, unsigned long long seed, int s0, long long t0, int amp,
                           const int16_t* wavs, int n_wavs, int wav_len, int every, void* stream) {
    hipLaunchKernelGGL(k_synth_pcm, dim3(4096), dim3(256), 0, (hipStream_t)stream, out, S, T, seed, s0, t0, amp, wavs,
                       n_wavs, wav_len, every);
    return ok(hipGetLastError());
}

int nnspk_launch_rfft(int32_t* x, int32_t* y, int n, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_rfft, dim3(n < 4096 ? n : 4096), dim3(64), 0, (hipStream_t)stream, x, y, n);
    return ok(hipGetLastError());
}

int nnspk_launch_pspec(int32_t* y, const int32_t* x, int len, int n, int shift, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_pspec, dim3((len + 255) / 256, n), dim3(256), 0, (hipStream_t)stream, y, x, len, n, shift);
    return ok(hipGetLastError());
}

int nnspk_launch_rfft_port(const int32_t* x, int32_t* y, int n, int cfft_only, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_rfft_port, dim3(n < 4096 ? n : 4096), dim3(64), 0, (hipStream_t)stream, x, y, n, cfft_only);
    return ok(hipGetLastError());
}

int nnspk_launch_fft_dif(int32_t* x, int32_t* y, int exp_nfft, int rfft, void* stream) {
    if (exp_nfft < 0 || exp_nfft > 8) return ok(hipErrorInvalidValue);
    hipLaunchKernelGGL(k_fft_dif, dim3(1), dim3(64), 0, (hipStream_t)stream, x, y, exp_nfft, rfft);
    return ok(hipGetLastError());
}

int nnspk_launch_cplx(int op, int32_t* o, int32_t* a, int32_t* b, int shift, int len, void* stream) {
    hipLaunchKernelGGL(k_cplx, dim3(1), dim3(64), 0, (hipStream_t)stream, op, o, a, b, shift, len, 0, 0);
    return ok(hipGetLastError());
}

int nnspk_launch_mel(const int32_t* spec, int32_t* mel, int n, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_mel, dim3((n * 40 + 255) / 256), dim3(256), 0, (hipStream_t)stream, spec, mel, n);
    return ok(hipGetLastError());
}

int nnspk_launch_log10(int32_t* out, const int32_t* x, int n, int add, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_log10, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, out, x, n, add);
    return ok(hipGetLastError());
}

int nnspk_launch_act(int type, const int32_t* x, void* y, int n, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_act, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, type, x, y, n);
    return ok(hipGetLastError());
}

int nnspk_launch_scalar(int op, const int32_t* in, int32_t* out, int n, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_scalar, dim3(op == 3 ? 1 : (n + 255) / 256), dim3(256), 0, (hipStream_t)stream, op, in, out, n);
    return ok(hipGetLastError());
}

int nnspk_launch_post(int nn_id, int thresh_prob, int th_count, void* post, int32_t* est, void* stream) {
    hipLaunchKernelGGL(k_post, dim3(1), dim3(64), 0, (hipStream_t)stream, nn_id, thresh_prob, th_count, post, est);
    return ok(hipGetLastError());
}

int nnspk_launch_fe_default(int16_t* prev5, int16_t* tail, const int32_t* mean, const int32_t* stdR,
                            int norm_shift, const uint8_t* mask, int n, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_fe_default, dim3((n * 40 + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       prev5, tail, mean, stdR, norm_shift, mask, n);
    return ok(hipGetLastError());
}

int nnspk_launch_nn_default(int16_t* h, int32_t* c, void* post, int row, const uint8_t* mask, int n,
                            void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_nn_default, dim3(n), dim3(64), 0, (hipStream_t)stream, h, c, post, row, mask, n);
    return ok(hipGetLastError());
}

// ---- thin runtime wrappers so the C host library needs no HIP headers -------
int nnspk_malloc(void** p, size_t n) { return ok(hipMalloc(p, n ? n : 16)); }
int nnspk_free(void* p) { return p ? ok(hipFree(p)) : 0; }
// fine-grained device memory the host writes directly (the drop-in workers'
// mailboxes and inputs), zeroed
int nnspk_malloc_finegrained(void** p, size_t n) {
    hipError_t e = hipExtMallocWithFlags(p, n, hipDeviceMallocFinegrained);
    if (e == hipSuccess) e = hipMemset(*p, 0, n);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    return ok(e);
}
int nnspk_memset(void* p, int v, size_t n, void* stream) { return ok(hipMemsetAsync(p, v, n, (hipStream_t)stream)); }
int nnspk_h2d(void* d, const void* h, size_t n, void* stream) {
    return ok(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, (hipStream_t)stream));
}
int nnspk_d2h(void* h, const void* d, size_t n, void* stream) {
    return ok(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, (hipStream_t)stream));
}
int nnspk_d2d(void* d, const void* s, size_t n, void* stream) {
    return ok(hipMemcpyAsync(d, s, n, hipMemcpyDeviceToDevice, (hipStream_t)stream));
}
int nnspk_sync(void* stream) { return ok(hipStreamSynchronize((hipStream_t)stream)); }
int nnspk_host_alloc(void** p, size_t n) { return ok(hipHostMalloc(p, n ? n : 16, hipHostMallocDefault)); }
int nnspk_host_free(void* p) { return p ? ok(hipHostFree(p)) : 0; }
int nnspk_host_alloc_mapped(void** p, void** dev, size_t n) {
    hipError_t e = hipHostMalloc(p, n ? n : 16, hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return ok(e);
    return ok(hipHostGetDevicePointer(dev, *p, 0));
}
int nnspk_stream_spin(void* stream) {
    for (;;) {
        const hipError_t r = hipStreamQuery((hipStream_t)stream);
        if (r == hipSuccess) return 0;
        if (r != hipErrorNotReady) return ok(r);
    }
}
int nnspk_stream_done(void* stream) {
    const hipError_t r = hipStreamQuery((hipStream_t)stream);
    return r == hipSuccess ? 1 : (r == hipErrorNotReady ? 0 : -ok(r));
}
int nnspk_event_sync(void* e) { return ok(hipEventSynchronize((hipEvent_t)e)); }
int nnspk_event_done(void* e) { return hipEventQuery((hipEvent_t)e) == hipSuccess; }
int nnspk_event_spin(void* e) {
    for (;;) {
        const hipError_t r = hipEventQuery((hipEvent_t)e);
        if (r == hipSuccess) return 0;
        if (r != hipErrorNotReady) return (int)r;
    }
}
int nnspk_device_count(int* n) { return ok(hipGetDeviceCount(n)); }
int nnspk_set_device(int d) { return ok(hipSetDevice(d)); }
int nnspk_get_device(int* d) { return ok(hipGetDevice(d)); }
const char* nnspk_error_string(int e) { return hipGetErrorString((hipError_t)e); }
int nnspk_stream_create(void** s) { return ok(hipStreamCreateWithFlags((hipStream_t*)s, hipStreamNonBlocking)); }
int nnspk_stream_create_prio(void** s, int high) {
    int least = 0, greatest = 0;
    hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
    if (e != hipSuccess) return ok(e);
    return ok(hipStreamCreateWithPriority((hipStream_t*)s, hipStreamNonBlocking, high ? greatest : least));
}
int nnspk_stream_destroy(void* s) { return s ? ok(hipStreamDestroy((hipStream_t)s)) : 0; }
int nnspk_event_create(void** e) { return ok(hipEventCreate((hipEvent_t*)e)); }
int nnspk_event_create_dep(void** e) { return ok(hipEventCreateWithFlags((hipEvent_t*)e, hipEventDisableTiming)); }
int nnspk_event_destroy(void* e) { return e ? ok(hipEventDestroy((hipEvent_t)e)) : 0; }
int nnspk_event_record(void* e, void* stream) { return ok(hipEventRecord((hipEvent_t)e, (hipStream_t)stream)); }
int nnspk_stream_wait(void* stream, void* event) {
    return ok(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)event, 0));
}
int nnspk_event_elapsed(float* ms, void* a, void* b) {
    return ok(hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b));
}
int nnspk_device_info(int* cus, int* clock_khz, char* name, int name_len) {
    int d = 0;
    hipDeviceProp_t p;
    int e = ok(hipGetDevice(&d));
    if (e) return e;
    e = ok(hipGetDeviceProperties(&p, d));
    if (e) return e;
    *cus = p.multiProcessorCount;
    *clock_khz = p.clockRate;
    if (name && name_len > 0) {
        int i = 0;
        for (; i < name_len - 1 && p.gcnArchName[i]; ++i) name[i] = p.gcnArchName[i];
        name[i] = 0;
    }
    return 0;
}

}  // extern "C"
