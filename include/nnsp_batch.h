/*
 * nnsp_batch.h -- batched multi-stream ns-nnsp on MI355X (libnnsp_mi355x.so).
 *
 * New fast path beside the drop-in single-stream API of nnsp_api.h: one
 * nnsp_batch runs NNSPClass_exec (reference ns-nnsp/src/nn_speech.c:74-127)
 * for S independent streams over a chunk of T frames per call, on one GPU.
 * Per stream and frame the result is bit-identical to calling the reference's
 * NNSPClass_exec on that stream's frames in order (same NeuralNetClass, same
 * accumulator width, same thresholds).
 *
 * Conventions (mirroring the reference): plain pointers and sizes, caller-owned
 * host buffers, integer return codes (0 = ok, <0 = argument error, >0 = HIP
 * error code, see nnsp_strerror).  The NeuralNetClass is only read during
 * nnsp_batch_create (weights, qbits, layer/activation functions are copied into
 * a device image); the LSTM state arrays it points to are not used by a batch.
 *
 * Layouts: pcm [S][T][160] int16 (stream-major chunk); trig [S][T] int16 =
 * NNSPClass_exec's return per frame; logits [S][T][nout] int32 = the NN output
 * on the frames where the NN ran (slides == 1), before post-processing
 * overwrites it (trap T7), and 0 on the other frames; features [S][T][40]
 * int16 = normFeatContext slot 5 per frame.
 */
#ifndef NNSP_BATCH_H
#define NNSP_BATCH_H
#include <stddef.h>
#include <stdint.h>

#include "nnsp_api.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct nnsp_batch nnsp_batch;

/* Per-stream post-processing state (NNSPClass fields slides..argmax_last). */
typedef struct {
    int16_t slides, trigger, argmax_last, pad0;
    int16_t counts_category[8];
    int16_t outputs[3], pad1;
} nnsp_post_state;

/* Creates a batch of n_streams on the current HIP device, all streams reset
 * (NNSPClass_reset).  nn_id selects post-processing as NNSPClass_exec does
 * (s2i_id -> s2i_post_proc, else binary_post_proc).  max_frames bounds T. */
int nnsp_batch_create(nnsp_batch **out, const NeuralNetClass *net, int nn_id,
                      const int32_t *mean, const int32_t *stdR, int16_t thresh_prob,
                      int16_t th_count, int n_streams, int max_frames);
/* The same for either build of the reference (ARM_OPTIMIZED, ambiq_nnsp_debug.h:4;
 * row N4 of SURVEY.md §8): arm_optimized = 1 is nnsp_batch_create (the shipped
 * build: CMSIS arm_rfft_q31 front end, interleaved weights, trap T1);
 * arm_optimized = 0 reproduces the reference compiled with ARM_OPTIMIZED=0:
 *   - front end: Frac15 window, fft.c's radix-4 DIF rfft, spec2pspec >> 15
 *     (spectrogram_module.c:33-77, feature_module.c:58-60);
 *   - net: weights in the portable byte order (affine.c:261-346: per 4-row
 *     block, per column pair, per row) and the live align shift before the bias
 *     (affine.c:311-313).  Returns NNSP_EUNSUPPORTED (see nnsp_strerror) for a
 *     layer whose align shift cannot be reproduced exactly (qbit_bias above
 *     qbit_input + qbit_kernel, or a sum that the shift could clamp). */
int nnsp_batch_create_ex(nnsp_batch **out, const NeuralNetClass *net, int nn_id,
                         const int32_t *mean, const int32_t *stdR, int16_t thresh_prob,
                         int16_t th_count, int n_streams, int max_frames, int arm_optimized);
void nnsp_batch_destroy(nnsp_batch *b);

/* NNSPClass_reset on the streams with mask[s] != 0 (mask == NULL: all). */
int nnsp_batch_reset(nnsp_batch *b, const uint8_t *mask);

/* Host-pointer chunk: copies pcm in, runs, copies the requested outputs back
 * (NULL skips an output) and synchronises. */
int nnsp_batch_exec(nnsp_batch *b, const int16_t *pcm, int T, int16_t *trig, int32_t *logits,
                    int16_t *features);

/* Device-pointer chunk, asynchronous on the batch's HIP stream.  pcm, trig and
 * logits are device pointers (trig / logits may be NULL). */
int nnsp_batch_exec_device(nnsp_batch *b, const int16_t *pcm, int T, int16_t *trig,
                           int32_t *logits);
int nnsp_batch_sync(nnsp_batch *b);
void *nnsp_batch_stream(nnsp_batch *b);           /* hipStream_t */
int nnsp_batch_streams(const nnsp_batch *b);      /* S */
int nnsp_batch_nout(const nnsp_batch *b);         /* width of the last layer */
const int16_t *nnsp_batch_features_device(const nnsp_batch *b); /* last chunk's [S][T][40] */

/* Device time of the last chunk's front-end and NN kernels (ms). */
int nnsp_batch_last_timing(nnsp_batch *b, float *fe_ms, float *nn_ms);

/* Post-processing state (outputs[3] etc.) of all streams -> host [S]. */
int nnsp_batch_post_state(nnsp_batch *b, nnsp_post_state *out);

/* Whole-stream state export / import (checkpoint / resume, or moving streams
 * between batches): nnsp_batch_state_bytes() bytes per stream. */
size_t nnsp_batch_state_bytes(const nnsp_batch *b);
int nnsp_batch_get_state(nnsp_batch *b, void *host, int first, int count);
int nnsp_batch_set_state(nnsp_batch *b, const void *host, int first, int count);

/* Synthetic PCM generator on the device (bench / tests): dev_out [S][T][160],
 * SplitMix64(seed, stream s0+s, sample t0*160+n) -> int16 in [-amp, amp-1]. */
int nnsp_synth_pcm(int16_t *dev_out, int S, int T, uint64_t seed, int s0, int64_t t0, int amp,
                   void *stream);
/* The same with recordings mixed in: stream g = s0 + s with
 * g % every == 0 replays dev_wavs[(g / every) % n_wavs][0 .. wav_len) (device
 * memory, n_wavs x wav_len int16) cyclically from sample offset
 * (g * 1601) % wav_len; the others are SplitMix64 as above. */
int nnsp_synth_pcm_mix(int16_t *dev_out, int S, int T, uint64_t seed, int s0, int64_t t0, int amp,
                       const int16_t *dev_wavs, int n_wavs, int wav_len, int every, void *stream);

/* Device selection / info (thin wrappers over the HIP runtime). */
int nnsp_device_count(int *n);
int nnsp_set_device(int dev);
int nnsp_device_info(int *compute_units, int *clock_khz, char *arch, int arch_len);
/* error codes (negative: argument / validation; positive: HIP runtime) */
#define NNSP_EINVAL (-1)
#define NNSP_EUNSUPPORTED (-2)
#define NNSP_ENOMEM (-3)
const char *nnsp_strerror(int code);

#ifdef __cplusplus
}
#endif
#endif
