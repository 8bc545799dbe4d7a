// nnsp_casc.h -- the cascade controller's per-frame logic and list bookkeeping
// (nnCntrlClass_exec, reference evb/src/nnCntrlClass.c:152-272), shared by
// casc_control_kernel (nnsp_cascade.hip) and the control stage fused into
// recur_pipe_kernel (nnsp_fast.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nnsp_kabi.h"

namespace nnsp {

// Append s to lists[n] for every lane with want; one atomic per wave and net.
// Every lane of the wave must call it (ballot).
__device__ __forceinline__ void list_push(int32_t* const* lists, int32_t* counts, int n, int s, bool want) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const bool mine = want && n == k;
        const unsigned long long m = __ballot(mine);
        if (!m) continue;
        const int leader = __ffsll((long long)m) - 1;
        int base = 0;
        if (lane == leader) base = atomicAdd(&counts[k], __popcll(m));
        base = __shfl(base, leader);
        if (mine) lists[k][base + __popcll(m & ((1ull << lane) - 1ull))] = s;
    }
}

// list s under net n for the next round; also on n's cold list while the
// net's STFT buffer still holds zeros from its reset (the front end runs in
// full for those frames)
__device__ __forceinline__ void list_next(const CascArgs& a, int n, int s, bool want, int fresh) {
    list_push(a.list, a.counts, n, s, want);
    list_push(a.cold_list, a.counts + 3, n, s, want && fresh < 2);
}

// frames scheduled per net: wave-reduce, one atomic per wave (whole wave calls)
__device__ __forceinline__ void add_frames(const CascArgs& a, int n, unsigned long long v) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        unsigned long long x = n == k ? v : 0ull;
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
        if ((threadIdx.x & 63) == 0 && x && a.frames) atomicAdd(&a.frames[k], x);
    }
}

// One frame of nnCntrlClass_exec for a stream running net n (the net at its
// sequence position) whose NNSPClass_exec returned det.  Updates the
// controller state; returns true when the frame resets net n (the stream's
// segment ends here and the next frame runs the net at st.pos from its reset).
// A move without a reset keeps the same net and state running.
// The counters and the position stay in range (0 <= cnt < timeout, 0 <= pos <
// len_seq: reset to 0, then only advanced here), so each "% m" of the
// reference is a compare-and-wrap: no integer division on the post wave.
__device__ __forceinline__ int wrap_inc(int x, int m) { return x + 1 == m ? 0 : x + 1; }
// a.seq[i] for a per-lane i, from the 2-bit packed copy (host, seq_bits).  A
// dynamic index into the kernel argument is a vector memory load, and its wait
// (vmcnt) also waited for the post wave's output stores issued just before.
__device__ __forceinline__ int seq_at(const CascArgs& a, int i) { return (a.seq_bits >> (2 * i)) & 3; }
__device__ __forceinline__ bool casc_step(const CascArgs& a, CascState& st, int n, int16_t det) {
    bool move = false, rst = false;
    int np = st.pos;
    if (n == 0) {   // s2i (nnCntrlClass.c:173-200)
        st.cnt_s2i = (uint16_t)wrap_inc(st.cnt_s2i, a.timeout_s2i);
        if (det || st.cnt_s2i == a.timeout_s2i - 1) {
            np = wrap_inc(st.pos, a.len_seq);
            move = true;
            if (det || n != seq_at(a, np)) {
                st.cnt_s2i = 0;
                rst = true;
            }
        }
    } else if (n == 2) {   // kws (nnCntrlClass.c:203-236)
        st.cnt_kws = (uint16_t)wrap_inc(st.cnt_kws, a.timeout_kws);
        if (det || st.cnt_kws == a.timeout_kws - 1) {
            np = det ? wrap_inc(st.pos, a.len_seq) : (st.pos == 0 ? a.len_seq - 1 : st.pos - 1);
            move = true;
            if (det || n != seq_at(a, np)) {
                st.cnt_kws = 0;
                rst = true;
            }
        }
    } else if (det) {   // vad (nnCntrlClass.c:238-262)
        np = wrap_inc(st.pos, a.len_seq);
        move = rst = true;
    }
    if (move) st.pos = (int16_t)np;
    return rst;
}

// casc_step for a wave-uniform net n with the per-lane decisions as selects:
// the branchy form put every per-lane condition behind exec-mask branches (the
// post wave of the binary nets ran ~200 scalar instructions per step, most of
// them exec-mask saves and restores).  Same state transitions as casc_step.
__device__ __forceinline__ bool casc_step_sel(const CascArgs& a, CascState& st, int n, int16_t det) {
    const int pos = st.pos;
    const int fwd = wrap_inc(pos, a.len_seq);
    if (n == 1) {   // vad (nnCntrlClass.c:238-262): a detection moves on and resets
        st.pos = (int16_t)(det ? fwd : pos);
        return det != 0;
    }
    const int to = n == 0 ? a.timeout_s2i : a.timeout_kws;
    const int cnt = wrap_inc(n == 0 ? st.cnt_s2i : st.cnt_kws, to);
    const bool move = det || cnt == to - 1;
    // s2i moves forward; kws forward on a detection, back on its timeout
    const int np = n == 0 || det ? fwd : (pos == 0 ? a.len_seq - 1 : pos - 1);
    const bool rst = move && (det || n != seq_at(a, np));
    const uint16_t c2 = (uint16_t)(rst ? 0 : cnt);
    if (n == 0)
        st.cnt_s2i = c2;
    else
        st.cnt_kws = c2;
    st.pos = (int16_t)(move ? np : pos);
    return rst;
}

// NNSPClass_reset's post-processing part (nn_speech.c:57-72)
template <class P>
__device__ __forceinline__ void post_reset(P& p) {
    p.slides = 1;
    p.trigger = 0;
    p.argmax_last = 0;
    for (int k = 0; k < 7; ++k) p.counts[k] = 0;
    p.outputs[0] = p.outputs[1] = p.outputs[2] = 0;
}

// segments cut by a net switch (one atomic per wave; whole wave calls)
__device__ __forceinline__ void count_cuts(const CascArgs& a, bool cut) {
    const unsigned long long m = __ballot(cut);
    if (m && a.cuts && (threadIdx.x & 63) == 0) atomicAdd(a.cuts, (int)__popcll(m));
}

// frames the next round schedules for a stream that continues at b_next
__device__ __forceinline__ unsigned long long next_frames(const CascArgs& a, int T, bool want, int b_next) {
    return want ? (unsigned long long)(a.seg_len > 0 ? min(a.seg_len, T - b_next) : T - b_next) : 0ull;
}

}  // namespace nnsp
