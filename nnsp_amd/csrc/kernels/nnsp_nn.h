// nnsp_nn.h -- shared NN building blocks (int8 MFMA with hi/lo activation
// planes, the affine_Krows fixed-point epilogue, activations, NNSPClass
// post-processing) used by the fused and the split NN kernels.
#pragma once
#include "nnsp_dev.h"
#include "nnsp_kabi.h"

namespace nnsp {

typedef int v4i __attribute__((ext_vector_type(4)));

// 16 int16 activations -> hi / lo' int8 planes: x = 256*hi + lo' + 128
__device__ __forceinline__ void split_hilo(const int16_t* p, v4i& hi, v4i& lo) {
    const int4 a = *reinterpret_cast<const int4*>(p);
    const int4 b = *reinterpret_cast<const int4*>(p + 8);
    const uint32_t HS = 0x07050301u, LS = 0x06040200u;
    hi.x = (int)__builtin_amdgcn_perm((uint32_t)a.y, (uint32_t)a.x, HS);
    hi.y = (int)__builtin_amdgcn_perm((uint32_t)a.w, (uint32_t)a.z, HS);
    hi.z = (int)__builtin_amdgcn_perm((uint32_t)b.y, (uint32_t)b.x, HS);
    hi.w = (int)__builtin_amdgcn_perm((uint32_t)b.w, (uint32_t)b.z, HS);
    lo.x = (int)(__builtin_amdgcn_perm((uint32_t)a.y, (uint32_t)a.x, LS) ^ 0x80808080u);
    lo.y = (int)(__builtin_amdgcn_perm((uint32_t)a.w, (uint32_t)a.z, LS) ^ 0x80808080u);
    lo.z = (int)(__builtin_amdgcn_perm((uint32_t)b.y, (uint32_t)b.x, LS) ^ 0x80808080u);
    lo.w = (int)(__builtin_amdgcn_perm((uint32_t)b.w, (uint32_t)b.z, LS) ^ 0x80808080u);
}

// the same from 16 int16 already in registers (a: elements 0..7, b: 8..15)
__device__ __forceinline__ void split_hilo_r(int4 a, int4 b, v4i& hi, v4i& lo) {
    const uint32_t HS = 0x07050301u, LS = 0x06040200u;
    hi.x = (int)__builtin_amdgcn_perm((uint32_t)a.y, (uint32_t)a.x, HS);
    hi.y = (int)__builtin_amdgcn_perm((uint32_t)a.w, (uint32_t)a.z, HS);
    hi.z = (int)__builtin_amdgcn_perm((uint32_t)b.y, (uint32_t)b.x, HS);
    hi.w = (int)__builtin_amdgcn_perm((uint32_t)b.w, (uint32_t)b.z, HS);
    lo.x = (int)(__builtin_amdgcn_perm((uint32_t)a.y, (uint32_t)a.x, LS) ^ 0x80808080u);
    lo.y = (int)(__builtin_amdgcn_perm((uint32_t)a.w, (uint32_t)a.z, LS) ^ 0x80808080u);
    lo.z = (int)(__builtin_amdgcn_perm((uint32_t)b.y, (uint32_t)b.x, LS) ^ 0x80808080u);
    lo.w = (int)(__builtin_amdgcn_perm((uint32_t)b.w, (uint32_t)b.z, LS) ^ 0x80808080u);
}

__device__ __forceinline__ v4i mfma8(v4i a, v4i b, v4i c) {
    return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ v4i load_frag(const uint8_t* base, int lane) {
    return *reinterpret_cast<const v4i*>(base + 16 * lane);
}

// Fixed-point epilogue of affine_Krows (is_out=1): exact sum + bias, shift,
// clamp (acc64) or wrap (acc32).  'pre' is the int64/int32 pre-bias value.
__device__ __forceinline__ int32_t affine_out(int64_t pre, int16_t b, const NnLayer& Ly, int acc32) {
    if (acc32) {
        int32_t s = (int32_t)pre;
        if (Ly.has_bias) s = wadd(s, Ly.bias_sh >= 0 ? wshl(b, Ly.bias_sh) : ((int32_t)b >> -Ly.bias_sh));
        return shift32(s, Ly.out_sh);
    }
    int64_t s = pre;
    if (Ly.has_bias) s += Ly.bias_sh >= 0 ? (int64_t)((uint64_t)(int64_t)b << Ly.bias_sh) : ((int64_t)b >> -Ly.bias_sh);
    return sat32(shift64(s, Ly.out_sh));
}

__device__ __forceinline__ int16_t act16(int act, int32_t v, const int16_t* tt) {
    return act == ACT_RELU6 ? relu6_q12(v) : (act == ACT_TANH ? tanh_q15(v, tt) : sigmoid_q15(v, tt));
}
// the same on the affine tables (act_q15; the split NN kernels' LDS copy at tb)
__device__ __forceinline__ int16_t act16s(int act, int32_t v, const uint8_t* tb) {
    return act == ACT_RELU6 ? relu6_q12(v) : (int16_t)(act == ACT_TANH ? act_q15<0>(v, tb) : act_q15<1>(v >> 1, tb));
}

// 8 features [8*part, 8*part + 8) of stream s at chunk frame t of a segment
// starting at b: from the net's feats buffer, or (cascade) from the net's
// ring of the shared front end's normalised output, except the 2 frames after
// a reset, which the cold front end wrote to feats
//
// The per-lane choice is a select of one address, not two branches with a
// load each: from the branchy form hipcc (ROCm 7.2) merged the two loads (and
// the caller's prev5 load) into one load whose base pointer it kept in an
// SGPR across the divergent branches, so the cold lanes of a wave read
// through another branch's base -- out of bounds, a memory fault in
// recur_pipe_kernel.  With the select the base is a VGPR per lane.
// fs.nring is wave-uniform.
// KNOWN: fr is the stream's fresh[] value, already loaded by the caller
// (proj's descriptor pipeline); otherwise it is loaded here for the first two
// frames of a segment
template <bool KNOWN = false>
__device__ __forceinline__ const int16_t* feat8_ptr(const FeatSrc& fs, const int16_t* feats, int s, int T, int b, int t,
                                                  int part, int fr = 2) {
    if (!fs.nring) return feats + ((size_t)s * T + t) * 40 + 8 * part;
    // only the first two frames of a segment can be cold: the fresh[] load
    // (and the dependent-load latency) only for those
    const bool cold = t - b < 2 && t - b + (KNOWN ? fr : (int)fs.fresh[s]) < 2;
    // (abs0 + t - lookback) mod ring with 0 <= abs0 < ring, 0 <= t < Tmax <=
    // ring and lookback < ring (host): the sum plus ring is in [1, 3 ring),
    // two conditional subtracts instead of a 32-bit division (~30 VALU)
    const unsigned rg = (unsigned)fs.ring;
    unsigned slot = (unsigned)(fs.abs0 + t - fs.lookback) + rg;
    slot = slot >= rg ? slot - rg : slot;
    slot = slot >= rg ? slot - rg : slot;
    const size_t row = cold ? (size_t)s * T + t : (size_t)s * fs.ring + slot;
    const uintptr_t base = cold ? (uintptr_t)feats : (uintptr_t)fs.nring;
    uintptr_t addr = base + (row * 40 + 8 * part) * sizeof(int16_t);
    // the address is opaque and lives in a VGPR pair: no compiler can
    // re-derive a wave-uniform (SGPR) base from the select above and merge
    // this load with another -- the hazard stays closed under a new hipcc, not
    // only under the ROCm 7.2 codegen it was found with
    asm volatile("" : "+v"(addr));
    return reinterpret_cast<const int16_t*>(addr);
}
__device__ __forceinline__ int4 feat8(const FeatSrc& fs, const int16_t* feats, int s, int T, int b, int t, int part) {
    return *reinterpret_cast<const int4*>(feat8_ptr(fs, feats, s, T, b, t, part));
}

// Preload the B fragments (hi, lo) of nkt k-tiles of a [16][stride] int16 buffer.
template <int MAXKT>
__device__ __forceinline__ void load_b(const int16_t* buf, int stride, int nkt, int lane,
                                       v4i (&bh)[MAXKT], v4i (&bl)[MAXKT]) {
    const int sc = lane & 15, q = lane >> 4;
#pragma unroll
    for (int kt = 0; kt < MAXKT; ++kt)
        if (kt < nkt) split_hilo(buf + sc * stride + 64 * kt + 16 * q, bh[kt], bl[kt]);
}

// Post-processing for one stream (nn_speech.c:146-227); lane-private state.
struct PostState {
    int16_t slides, trigger, argmax_last, pad0;
    int16_t counts[8];
    int16_t outputs[3], pad1;
};

template <typename LG>
__device__ __forceinline__ int argmax_lw(const LG& v, int n, int off = 0) {
    int am = 0;
    int32_t m = v[off];
    for (int i = 1; i < n; ++i)
        if (v[off + i] >= m) { m = v[off + i]; am = i; }
    return am;
}

// logits view over an LDS row: int32 (linear last layer) or int16
struct LogitRow {
    const int16_t* p;
    bool lin;
    __device__ __forceinline__ int32_t operator[](int i) const {
        return lin ? reinterpret_cast<const int32_t*>(p)[i] : (int32_t)p[i];
    }
};

// s2i_post_proc (nn_speech.c:191-227) with its logits in an LDS row (16-byte
// aligned): the 7 intent logits come in with two 16-byte loads; the two
// 17-way slot argmaxes read LDS only on a detection.  Same results as
// post_proc's s2i branch.
__device__ __forceinline__ void post_proc_s2i_lds(PostState& ps, const NnImage& img, const int32_t* f32) {
    const int4 a = *reinterpret_cast<const int4*>(f32);
    const int4 b = *reinterpret_cast<const int4*>(f32 + 4);
    const int32_t v[7] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z};
    ps.trigger = 0;
    ps.outputs[0] = ps.outputs[1] = ps.outputs[2] = 0;
    int am = 0;
    int32_t m = v[0];
#pragma unroll
    for (int i = 1; i < 7; ++i)
        if (v[i] >= m) { m = v[i]; am = i; }
    if (ps.argmax_last == 0 || ps.argmax_last == am) {
        if (am != 0) {
            int16_t cam = 0;
#pragma unroll
            for (int i = 1; i < 7; ++i)
                if (i == am) {
                    ps.counts[i] = (int16_t)(ps.counts[i] + 1);
                    cam = ps.counts[i];
                }
            if (cam > img.th_count) {
                ps.trigger = 1;
                ps.outputs[0] = (int16_t)am;
                ps.outputs[1] = (int16_t)argmax_lw(f32, 17, 7);
                ps.outputs[2] = (int16_t)argmax_lw(f32, 17, 24);
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < 7; ++i) ps.counts[i] = 0;
    }
    ps.argmax_last = (int16_t)am;
}

// binary_post_proc (nn_speech.c:193-227; T7: logits overwritten by exp2 values)
template <typename LG>
__device__ __forceinline__ void post_proc_binary(PostState& ps, const NnImage& img, const LG& lg) {
    // the larger logit's difference to the max is 0, and compute_pwr2(0)
    // is the constant 32723 (0x5a82 + 0x1fd7 + 0x057a): only the other
    // logit's exp2 is computed -- the post wave is the slowest stage of
    // the binary nets' recurrence pipeline
    const int32_t l0 = lg[0], l1 = lg[1];
    const bool first = l0 >= l1;   // on a tie both differences are 0
    const int32_t eo = pwr2_q15(sat32(((int64_t)(first ? wsub(l1, l0) : wsub(l0, l1)) * 0xB8AA) >> 15));
    const int32_t e[2] = {first ? 32723 : eo, first ? eo : 32723};
    const int32_t den = wadd(e[0], e[1]);
    const int32_t lim = (int32_t)(((int64_t)(32768 - img.thresh_prob) * den) >> 15);
    ps.counts[0] = e[0] <= lim ? (int16_t)(ps.counts[0] + 1) : (int16_t)0;
    ps.trigger = ps.counts[0] >= img.th_count ? 1 : 0;
}

template <typename LG>
__device__ __forceinline__ void post_proc(PostState& ps, const NnImage& img, const LG& lg) {
    if (img.nn_id == 0) {  // s2i_post_proc
        ps.trigger = 0;
        ps.outputs[0] = ps.outputs[1] = ps.outputs[2] = 0;
        const int am = argmax_lw(lg, 7);
        if (ps.argmax_last == 0 || ps.argmax_last == am) {
            if (am != 0) {
                // counts[am]++ without a runtime register index (keeps ps in VGPRs)
                int16_t cam = 0;
#pragma unroll
                for (int i = 1; i < 7; ++i)
                    if (i == am) {
                        ps.counts[i] = (int16_t)(ps.counts[i] + 1);
                        cam = ps.counts[i];
                    }
                if (cam > img.th_count) {
                    ps.trigger = 1;
                    ps.outputs[0] = (int16_t)am;
                    ps.outputs[1] = (int16_t)argmax_lw(lg, 17, 7);
                    ps.outputs[2] = (int16_t)argmax_lw(lg, 17, 24);
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < 7; ++i) ps.counts[i] = 0;
        }
        ps.argmax_last = (int16_t)am;
    } else {
        post_proc_binary(ps, img, lg);
    }
}


}  // namespace nnsp
