// nnsp_cascade.hip -- control kernels of the batched VAD -> KWS -> S2I cascade
// (nnCntrlClass_exec, reference evb/src/nnCntrlClass.c:152-272).
//
// A chunk of T frames runs in rounds.  In a round every still-running stream
// executes ONE net (the one at its current sequence position) speculatively
// from its segment start to the end of the chunk (proj/recur/fe kernels with a
// stream list).  casc_control_kernel then replays the controller's per-frame
// logic over that segment's triggers: timeout counters, detection, the next
// sequence position and the NNSPClass_reset of the departing net.  At the first
// frame that moves the stream to a different net state, the segment is cut:
// the departing net is reset (its normFeatContext slot 5 keeps the feature of
// that frame -- FeatureClass_setDefault leaves slot 5 alone, trap T4) and the
// stream is listed for the next round from the following frame.  Everything
// the departing net computed past the cut is discarded by the reset.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "nnsp_kabi.h"
#include "nnsp_casc.h"
#include "nnsp_nn.h"

using nnsp::feat8;

namespace {

using nnsp::add_frames;
using nnsp::list_next;

inline int ok(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }

// Round 0's lists: every stream under the net at its sequence position.  The
// appends are aggregated per 1024-thread workgroup (one global atomic per list
// and workgroup, 9 in all): per-wave atomics on the same six counters (4 600
// for 32 768 streams) serialised at the L2 and took ~40 us.
__global__ __launch_bounds__(1024) void casc_begin_kernel(CascArgs a) {
    __shared__ int wcnt[16][6];   // per wave: entries for list k (k < 3) and cold list k - 3
    __shared__ int gbase[6];
    __shared__ unsigned long long fsum[3];
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nwv = blockDim.x >> 6;
    const bool ok_s = s < a.S;
    int n = 0, fr = 2;
    if (ok_s) {
        a.seg_begin[s] = 0;
        n = nnsp::seq_at(a, a.st[s].pos);
        fr = a.fresh[s];
    }
    unsigned long long m[6];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        m[k] = __ballot(ok_s && n == k);
        m[k + 3] = __ballot(ok_s && n == k && fr < 2);
    }
    if (lane == 0)
#pragma unroll
        for (int j = 0; j < 6; ++j) wcnt[w][j] = __popcll(m[j]);
    if (threadIdx.x < 3) fsum[threadIdx.x] = 0ull;
    __syncthreads();
    if (threadIdx.x < 6) {   // exclusive prefix over the waves, one global atomic per list
        const int j = threadIdx.x;
        int tot = 0;
        for (int q = 0; q < nwv; ++q) {
            const int c = wcnt[q][j];
            wcnt[q][j] = tot;
            tot += c;
        }
        gbase[j] = tot ? atomicAdd(&a.counts[j], tot) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 6; ++j)
        if ((m[j] >> lane) & 1ull) {
            int32_t* lst = j < 3 ? a.list[j] : a.cold_list[j - 3];
            lst[gbase[j] + wcnt[w][j] + __popcll(m[j] & ((1ull << lane) - 1ull))] = s;
        }
    // frames scheduled per net (statistics): wave sums, then one atomic per net
    const unsigned long long v = ok_s ? (unsigned long long)(a.seg_len > 0 ? min(a.seg_len, a.T) : a.T) : 0ull;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        unsigned long long x = n == k ? v : 0ull;
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
        if (lane == 0 && x) atomicAdd(&fsum[k], x);
    }
    __syncthreads();
    if (threadIdx.x < 3 && fsum[threadIdx.x] && a.frames) atomicAdd(&a.frames[threadIdx.x], fsum[threadIdx.x]);
}

__global__ __launch_bounds__(256) void casc_control_kernel(CascArgs a) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < 6 && a.counts_clear) a.counts_clear[s] = 0;
    const int T = a.T;
    bool want = false, was_cut = false;
    int n_next = 0, b_next = T, fr_next = 2;
    if (s < a.S && a.seg_begin[s] < T) {
        const int b = a.seg_begin[s];
        const int e = a.seg_len > 0 ? min(T, b + a.seg_len) : T;   // this round's segment b..e-1
        CascState st = a.st[s];
        const int n = a.seq[st.pos];   // the net that ran this round (fixed over the segment)
        const int16_t* tr = a.trig[n] + (size_t)s * T;
        int cut = -1;
        b_next = e;   // no switch: carry on in the same net next round (if e < T)
        // the caller's per-frame outputs were written by the net's recur kernel;
        // here only the controller runs, 16 prefetched triggers at a time
        int16_t dq[16];
        for (int t = b; t < e; ++t) {
            if (((t - b) & 15) == 0) {
#pragma unroll
                for (int k = 0; k < 16; ++k) dq[k] = t + k < e ? tr[t + k] : (int16_t)0;
            }
            const int16_t det = dq[(t - b) & 15];
            const bool rst = nnsp::casc_step(a, st, n, det);
            if (rst) {
                cut = t;
                break;
            }
        }
        // frames since the reset of the net the stream runs next round (the
        // front end's STFT buffer is zero right after NNSPClass_reset)
        fr_next = cut >= 0 ? 0 : min(2, (int)a.fresh[s] + (e - b));
        int4 slot5[5];   // the cut frame's feature, read while fresh[s] is still the segment's
        if (cut >= 0)
#pragma unroll
            for (int k = 0; k < 5; ++k) slot5[k] = feat8(a.fs[n], a.feats[n], s, T, b, cut, k);
        a.fresh[s] = (int8_t)fr_next;
        if (cut >= 0) {
            // NNSPClass_reset of the departing net (nn_speech.c:57-72):
            // FeatureClass_setDefault -- context slots 0..4 := the default,
            // slot 5 keeps this frame's feature (T4); the STFT buffer's zeros
            // are fresh = 0 of the next net to run -- then the LSTM state
            // (NeuralNetClass_setDefault) and the post-processing state
            const int4* def = reinterpret_cast<const int4*>(a.prev_default[n]);
            int4* p5 = reinterpret_cast<int4*>(a.prev5[n] + (size_t)s * 200);
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                const int4 d = def[k];
                p5[k] = d;
                p5[5 + k] = d;
                p5[10 + k] = d;
                p5[15 + k] = d;
                p5[20 + k] = slot5[k];
            }
            const int4 z = make_int4(0, 0, 0, 0);
            int4* hs = reinterpret_cast<int4*>(a.h[n] + (size_t)s * NN_MAX_W);
            int4* cs = reinterpret_cast<int4*>(a.c[n] + (size_t)s * NN_MAX_W);
            for (int k = 0; k < NN_MAX_W / 8; ++k) hs[k] = z;
            for (int k = 0; k < NN_MAX_W / 4; ++k) cs[k] = z;
            nnsp::post_reset(*(reinterpret_cast<NnPost*>(a.post[n]) + s));
            b_next = cut + 1;
            was_cut = true;
        }
        a.st[s] = st;
        a.seg_begin[s] = b_next;
        if (b_next < T) {
            want = true;
            n_next = nnsp::seq_at(a, st.pos);
        }
    }
    list_next(a, n_next, s, want, fr_next);
    if (a.last_round && __ballot(want) && (threadIdx.x & 63) == 0) atomicMax(a.last_round, a.round + 1);
    add_frames(a, n_next, nnsp::next_frames(a, T, want, b_next));
    nnsp::count_cuts(a, was_cut);
}

// nnCntrlClass_reset's controller part + PcmBufClass_reset (nnCntrlClass.c:132-150,
// PcmBufClass.c:19-28): timeout counters, the PCM history and the shared
// front end's PCM tail; every net restarts from its reset (fresh 0).  The
// sequence position is kept, as the reference does.
__global__ __launch_bounds__(256) void casc_reset_kernel(CascState* st, int16_t* hist, int H, int16_t* stail,
                                                        int8_t* fresh, const uint8_t* mask, int S) {
    const int s = blockIdx.x;
    if (s >= S || (mask && !mask[s])) return;
    if (threadIdx.x == 0) {
        st[s].cnt_kws = 0;
        st[s].cnt_s2i = 0;
        fresh[s] = 0;
    }
    int4* h = reinterpret_cast<int4*>(hist + (size_t)s * H * 160);
    for (int i = threadIdx.x; i < H * 20; i += blockDim.x) h[i] = make_int4(0, 0, 0, 0);
    int4* tl = reinterpret_cast<int4*>(stail + (size_t)s * 320);
    for (int i = threadIdx.x; i < 40; i += blockDim.x) tl[i] = make_int4(0, 0, 0, 0);
}

// dst := last H frames of (src ++ pcm chunk), per stream (int4 = 8 samples).
__global__ __launch_bounds__(256) void hist_roll_kernel(int16_t* dst, const int16_t* src, const int16_t* pcm, int S,
                                                       int T, int H) {
    const long long n = (long long)S * H * 20;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const int s = (int)(i / (H * 20));
        const int r = (int)(i - (long long)s * H * 20);
        const int k = r / 20, c = r % 20;   // history frame k, chunk c
        const int j = T + k;                // index into src(H) ++ pcm(T)
        const int4* p = j < H ? reinterpret_cast<const int4*>(src + ((size_t)s * H + j) * 160) + c
                              : reinterpret_cast<const int4*>(pcm + ((size_t)s * T + j - H) * 160) + c;
        reinterpret_cast<int4*>(dst + ((size_t)s * H + k) * 160)[c] = *p;
    }
}

// Per-stream state blobs (StateCopy, nnsp_kabi.h): one workgroup per stream,
// its threads over each segment's bytes -- dwords when the row and both ends
// are 4-byte aligned (all but the controller's 1-byte frames-since-reset).
__global__ __launch_bounds__(256) void state_copy_kernel(StateCopy sc, uint8_t* blob) {
    for (int i = blockIdx.x; i < sc.count; i += gridDim.x) {
        const unsigned long long s = (unsigned long long)(sc.first + i);
        uint8_t* b = blob + (size_t)i * sc.per;
        for (int k = 0; k < sc.nseg; ++k) {
            const StateSeg& g = sc.seg[k];
            const bool w4 = ((g.row_bytes | g.off | g.base | g.stride | g.row_pitch) & 3) == 0;
            const uint32_t unit = w4 ? 4 : 1, per_row = g.row_bytes / unit;
            for (uint32_t u = threadIdx.x; u < g.rows * per_row; u += blockDim.x) {
                const uint32_t r = u / per_row, o = (u - r * per_row) * unit;
                uint8_t* dev = reinterpret_cast<uint8_t*>(g.base + s * g.stride +
                                                          (unsigned long long)((g.row0 + r) % g.wrap) * g.row_pitch) + o;
                uint8_t* bl = b + g.off + (size_t)r * g.row_bytes + o;
                if (w4) {
                    if (sc.to_blob)
                        *reinterpret_cast<uint32_t*>(bl) = *reinterpret_cast<const uint32_t*>(dev);
                    else
                        *reinterpret_cast<uint32_t*>(dev) = *reinterpret_cast<const uint32_t*>(bl);
                } else {
                    if (sc.to_blob)
                        *bl = *dev;
                    else
                        *dev = *bl;
                }
            }
        }
    }
}

}  // namespace

extern "C" {

int nnspk_launch_state_copy(const StateCopy* sc, void* blob, void* stream) {
    if (sc->count <= 0) return 0;
    if (sc->nseg < 0 || sc->nseg > NNSP_STATE_SEGS) return ok(hipErrorInvalidValue);
    for (int k = 0; k < sc->nseg; ++k)
        if (!sc->seg[k].wrap || sc->seg[k].off + (unsigned long long)sc->seg[k].rows * sc->seg[k].row_bytes > sc->per)
            return ok(hipErrorInvalidValue);
    const int blocks = sc->count < 4096 ? sc->count : 4096;
    hipLaunchKernelGGL(state_copy_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, *sc, (uint8_t*)blob);
    return ok(hipGetLastError());
}

int nnspk_launch_casc_begin(const CascArgs* a, void* stream) {
    if (a->S <= 0) return 0;
    hipLaunchKernelGGL(casc_begin_kernel, dim3((a->S + 1023) / 1024), dim3(1024), 0, (hipStream_t)stream, *a);
    return ok(hipGetLastError());
}

int nnspk_launch_casc_control(const CascArgs* a, void* stream) {
    if (a->S <= 0) return 0;
    hipLaunchKernelGGL(casc_control_kernel, dim3((a->S + 255) / 256), dim3(256), 0, (hipStream_t)stream, *a);
    return ok(hipGetLastError());
}

int nnspk_launch_casc_reset(CascState* st, int16_t* hist, int hist_frames, int16_t* stail, int8_t* fresh,
                            const uint8_t* mask, int S, void* stream) {
    if (S <= 0) return 0;
    hipLaunchKernelGGL(casc_reset_kernel, dim3(S), dim3(256), 0, (hipStream_t)stream, st, hist, hist_frames, stail,
                       fresh, mask, S);
    return ok(hipGetLastError());
}

int nnspk_launch_hist_roll(int16_t* dst, const int16_t* src, const int16_t* pcm, int S, int T, int hist_frames,
                           void* stream) {
    if (S <= 0 || hist_frames <= 0) return 0;
    const long long n = (long long)S * hist_frames * 20;
    long long blocks = (n + 255) / 256;
    if (blocks > 256 * 32) blocks = 256 * 32;
    hipLaunchKernelGGL(hist_roll_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, dst, src, pcm,
                       S, T, hist_frames);
    return ok(hipGetLastError());
}

}  // extern "C"
