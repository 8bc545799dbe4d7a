/*
 * nnsp_cascade.h -- batched VAD -> KWS -> S2I cascade on MI355X
 * (libnnsp_mi355x.so).
 *
 * The batched counterpart of the reference's nnCntrlClass
 * (evb/src/nnCntrlClass.h:35-58, nnCntrlClass.c:57-272): per stream, every
 * 10 ms frame goes to the net at the stream's current sequence position; a
 * VAD detection moves on to the next position; KWS moves forward on a
 * detection and back on its timeout; S2I moves on after a detection or its
 * timeout.  The departing net is reset (NNSPClass_reset) on each move.  KWS and
 * S2I read the PCM frame that lies frs_vbufBk frames in the past (PcmBufClass,
 * 100-frame voice buffer).
 *
 * A cascade drives three nnsp_batch objects of the same stream count, indexed
 * by NNSP_ID (s2i_id = 0, vad_id = 1, kws_galaxy_id = 2,
 * nnsp_identification.h).  Their thresholds come from the batches
 * (nnsp_batch_create).  Per stream and frame, the net that ran, the trigger it
 * returned and NNSPClass.outputs are bit-identical to calling the reference's
 * nnCntrlClass_exec on that stream's frames in order.
 */
#ifndef NNSP_CASCADE_H
#define NNSP_CASCADE_H
#include <stdint.h>

#include "nnsp_batch.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct nnsp_cascade nnsp_cascade;

/* The ParamCntrlClass fields (nnCntrlClass.h:12-31) that the nets do not
 * already carry: look-back frames and timeouts of S2I and KWS. */
typedef struct {
    int16_t frs_vbufBk_s2i;      /* 0..99 */
    int16_t thresh_timeout_s2i;  /* >= 1 */
    int16_t frs_vbufBk_kws;      /* 0..99 */
    int16_t thresh_timeout_kws;  /* >= 1 */
} nnsp_cascade_params;

/* nnCntrlClass_init: nets[NNSP_ID] (all with the same n_streams and a
 * max_frames the chunks will not exceed), seq = NNSP_ID per sequence position
 * (pt_seq_cntrl, len 1..8).  Every stream starts at position 0 with all nets
 * reset.  The nets stay owned by the caller and must outlive the cascade;
 * their HIP streams (nnsp_batch_stream) carry the nets' rounds, so a batch of
 * a cascade must not be run on its own while the cascade is in use. */
int nnsp_cascade_create(nnsp_cascade **out, nnsp_batch *const nets[3], const int8_t *seq,
                        int len_seq, const nnsp_cascade_params *params);
void nnsp_cascade_destroy(nnsp_cascade *c);

/* nnCntrlClass_reset on the streams with mask[s] != 0 (NULL: all): timeout
 * counters, all three nets and the PCM history; the position is kept. */
int nnsp_cascade_reset(nnsp_cascade *c, const uint8_t *mask);

/* One chunk of T frames: pcm [S][T][160] int16.  Outputs per frame (NULL
 * skips): net_ran [S][T] int8 = NNSP_ID that ran, detected [S][T] int16 = its
 * NNSPClass_exec return, outputs3 [S][T][3] int16 = its NNSPClass.outputs.
 * _device: device pointers, work on nnsp_cascade_stream and the three nets'
 * batch streams forked from it.  The call returns once the chunk's rounds have
 * finished on the device (its outputs are final): the host reads back the list
 * lengths of the round after the last one it launched to decide whether more
 * rounds are needed, so it cannot queue the next chunk while this one runs.
 * The chunk's counters come back with that read; its bookkeeping (clearing
 * them, the next chunk's STFT tail and look-back history, a look-ahead front
 * end) may still run on
 * nnsp_cascade_stream when it returns; the next call, the statistics getters,
 * nnsp_cascade_sync and nnsp_cascade_reset order themselves after it. */
int nnsp_cascade_exec(nnsp_cascade *c, const int16_t *pcm, int T, int8_t *net_ran,
                      int16_t *detected, int16_t *outputs3);
int nnsp_cascade_exec_device(nnsp_cascade *c, const int16_t *pcm, int T, int8_t *net_ran,
                             int16_t *detected, int16_t *outputs3);
/* The same, plus a look-ahead: next_pcm (device, [S][next_T][160]) is the
 * chunk the NEXT call will receive.  Its shared front end (the log-Mel of
 * every frame, about half a chunk's device time) is queued behind this chunk's
 * controller start and runs while the nets' rounds of this chunk run, so the
 * two overlap.  The next call skips its own front end when it receives exactly
 * that pointer and T; next_pcm must hold its final samples when passed and stay
 * unchanged until then (nnsp_cascade_reset drops the look-ahead).  Used when
 * the nets run concurrently (not in serial mode) and T, next_T >= the
 * look-back + 1; otherwise it is ignored.  Results are identical.  next_pcm is
 * read by the look-ahead front end until this call returns; with the
 * development mode NNSP_EARLY_RETURN=1 (the call returns once the rounds are
 * done) it is read until the next call on this cascade, nnsp_cascade_sync or
 * nnsp_cascade_reset returns. */
int nnsp_cascade_exec_device_ahead(nnsp_cascade *c, const int16_t *pcm, int T, const int16_t *next_pcm,
                                   int next_T, int8_t *net_ran, int16_t *detected, int16_t *outputs3);
int nnsp_cascade_sync(nnsp_cascade *c);

/* Scheduling knob (results do not depend on it): each round runs every
 * listed stream for at most this many frames (0: to the chunk end).  Smaller
 * windows waste less work past a net switch but take more rounds.  -1
 * (default): chosen per chunk from the previous chunk's net switches per
 * stream (< 0.5: 0, < 2: 32, else 16; the first chunk uses 16).  The
 * environment NNSP_CASCADE_WINDOW (>= 0) fixes it at create time. */
int nnsp_cascade_set_window(nnsp_cascade *c, int frames);
/* The window the next chunk will use, whether it is automatic, and the
 * number of segments the last chunk cut at a net switch. */
int nnsp_cascade_get_window(nnsp_cascade *c, int *frames, int *is_auto, int *last_cuts);
void *nnsp_cascade_stream(nnsp_cascade *c);

/* Last chunk: rounds run, frames scheduled on the nets (>= S*T; the excess is
 * work past a switch that the switch discarded), device time in ms. */
int nnsp_cascade_last_stats(nnsp_cascade *c, int *rounds, long long *frames_run, float *ms);

/* Per-round, per-net device timing (HIP events around each net's work in
 * every round) for nnsp_cascade_last_net_stats.  Off by default: the events
 * cost a few percent of throughput (environment NNSP_CASCADE_TIMING=1 turns
 * it on at create time). */
int nnsp_cascade_set_timing(nnsp_cascade *c, int on);

/* Instrumentation: on = the three nets' work of each round runs one net after
 * the other on the cascade's own stream instead of concurrently on three
 * forked streams (environment NNSP_CASCADE_SERIAL at create time).  With timing
 * on, the per-net event spans then time each net's kernels alone.  Results do
 * not depend on it. */
int nnsp_cascade_set_serial(nnsp_cascade *c, int on);

/* Last chunk, one net (NNSP_ID): frames scheduled on it, the device time of
 * the front end of the frames right after its resets and of its NN kernels
 * (proj + recur, the controller fused in) summed over the rounds (0 unless
 * timing is on), and the number of rounds it ran in (one launch of each
 * kernel per round). */
int nnsp_cascade_last_net_stats(nnsp_cascade *c, int nn_id, long long *frames_run, float *fe_ms,
                                float *nn_ms, int *launches);

/* Last chunk: device time in ms of the shared front end (the log-Mel of every
 * frame of every stream, one launch; timed in the previous call when that call
 * ran it ahead). */
int nnsp_cascade_last_fe_stats(nnsp_cascade *c, float *ms);

/* Last chunk, per round k < max_rounds and net i (NNSP_ID): the number of
 * streams listed ([3k + i] of lists) and, when timing is on, the device ms of
 * the net's cold-frame front end and NN kernels in that round (else 0).  Any
 * output may be NULL.  Returns the number of rounds recorded (at most 32), or
 * a negative error code. */
int nnsp_cascade_last_rounds(nnsp_cascade *c, int max_rounds, int32_t *lists, float *fe_ms, float *nn_ms);

/* Running totals since create or the last nnsp_cascade_totals_reset, for a
 * caller that times many chunks and reads statistics once afterwards: chunks
 * taken, rounds, frames scheduled on the nets, the shared front end's device
 * ms, and the device ms from each chunk's start to its rounds' end.  Any
 * output may be NULL; a chunk counts once its counters are taken (the next
 * call, a getter or nnsp_cascade_sync). */
int nnsp_cascade_totals(nnsp_cascade *c, long long *chunks, long long *rounds, long long *frames_run,
                        double *fe_ms, double *chunk_ms);
int nnsp_cascade_totals_reset(nnsp_cascade *c);

/* current_pos_seq of every stream -> host int8 [S]. */
int nnsp_cascade_positions(nnsp_cascade *c, int8_t *pos);

/* Whole-stream state export / import between chunks: checkpoint / resume, or
 * moving streams between cascades (shards) of the same nets and parameters.
 * One blob of nnsp_cascade_state_bytes() bytes per stream holds what the
 * reference keeps per stream -- one nnCntrlClass, its PcmBufClass and the
 * three NNSPClass / FeatureClass / NeuralNetClass states
 * (evb/src/nnCntrlClass.h:35-45, PcmBufClass.h:9-16, nn_speech.h):
 *
 *   nnsp_cascade_stream_hdr                       32 B (below)
 *   PCM history  int16 [H][160]   the stream's last H frames, oldest first
 *                                 (PcmBufClass's voice buffer as far back as
 *                                 the look-backs reach, and the STFT buffer of
 *                                 a net at the largest one: H = max(frs_vbufBk) + 2)
 *   STFT tail    int16 [320]      the last two frames (the shared front end's
 *                                 stftModule.dataBuffer before the next frame)
 *   look-back features int16 [3][H - 2][40]   per NNSP_ID, the normalised
 *                                 log-Mel of frames -(H-2) .. -1, which KWS and
 *                                 S2I read frs_vbufBk frames back
 *   3 x nnsp_batch blob           per NNSP_ID, nnsp_batch_get_state's layout:
 *                                 that net's STFT tail, normFeatContext slots
 *                                 1..5, LSTM h and c, post-processing state
 *
 * get waits for the cascade's work; set drops a look-ahead front end (the next
 * call recomputes its own).  Blobs carry H, their size and a signature of the
 * three nets' state shapes (LSTM width and layers, outputs); set refuses blobs
 * of a cascade with other look-backs or other nets (NNSP_EINVAL). */
typedef struct {
    uint32_t magic;               /* NNSP_CASCADE_STATE_MAGIC */
    uint16_t hist_frames;         /* H */
    uint16_t version;             /* 1 */
    int16_t current_pos_seq;      /* nnCntrlClass */
    uint16_t cnt_timeout_kws;
    uint16_t cnt_timeout_s2i;
    int16_t reserved0;
    int8_t frames_since_reset;    /* frames the current net ran since its reset (0, 1, 2 = 2 or more) */
    int8_t reserved1[3];
    uint32_t state_bytes;         /* nnsp_cascade_state_bytes() of the cascade that wrote it */
    uint32_t nets_sig;            /* FNV-1a of each net's state shape (NNSP_ID order) */
    uint32_t reserved2;
} nnsp_cascade_stream_hdr;
#define NNSP_CASCADE_STATE_MAGIC 0x3153434eu   /* "NCS1" */
#define NNSP_CASCADE_STATE_VERSION 2
size_t nnsp_cascade_state_bytes(const nnsp_cascade *c);
int nnsp_cascade_get_state(nnsp_cascade *c, void *host, int first, int count);
int nnsp_cascade_set_state(nnsp_cascade *c, const void *host, int first, int count);

/* Stream state in the reference's own per-stream objects: moving a live
 * single-stream session of the reference (one nnCntrlClass, its PcmBufClass
 * and three NNSPClass) onto the batched cascade and back.
 *
 * The EVB controller's structs are not part of ns-nnsp's API; these are
 * ABI-identical mirrors (evb/src/nnCntrlClass.h:11-45, PcmBufClass.h:9-16):
 * an application passes pointers to its own nnCntrlClass / PcmBufClass cast
 * to them. */
typedef struct {
    int16_t thresh_prob_vad, thresh_cnts_vad;
    int16_t frs_vbufBk_s2i, thresh_timeout_s2i, thresh_prob_s2i, thresh_cnts_s2i;
    int16_t frs_vbufBk_kws, thresh_timeout_kws, thresh_prob_kws, thresh_cnts_kws;
} nnsp_ref_params;                /* ParamCntrlClass */
typedef struct {
    void *pt_seq_cntrl;
    int8_t len_seq_cntrl;
    int8_t current_pos_seq;
    void *pt_nnsp_arry;
    nnsp_ref_params Params;
    uint16_t cnt_timeout_kws;
    uint16_t cnt_timeout_s2i;
    uint16_t cnt_voice_frames_detected;
    uint16_t cnt_voice_frames_not_detected;
} nnsp_ref_cntrl;                 /* nnCntrlClass */
typedef struct {
    int16_t *pcm_buffer;          /* [num_frs][smpls_fr] */
    int16_t idx_set;
    int16_t idx_data_latest;
    int16_t num_frs;
    int16_t smpls_fr;
} nnsp_ref_pcmbuf;                /* PcmBufClass */

/* One stream: its controller, voice buffer and the three NNSPClass by
 * NNSP_ID (nnsp[i]->pt_feat: its FeatureClass; nnsp[i]->pt_net: its
 * NeuralNetClass, whose LSTM layers' pt_hstate / pt_cstate hold the state). */
typedef struct {
    nnsp_ref_cntrl *cntrl;
    nnsp_ref_pcmbuf *pcmbuf;
    NNSPClass *nnsp[3];
} nnsp_ref_stream;

/* set_state_ref: streams first .. first + count - 1 take the state the
 * reference objects refs[i] hold between two nnCntrlClass_exec calls.  Read:
 * current_pos_seq and the two timeout counters; the voice buffer's frames as
 * far back as the look-backs reach (from idx_data_latest; smpls_fr 160,
 * num_frs >= max(frs_vbufBk) + 1); per net its post-processing state
 * (slides, trigger, counts_category, outputs, argmax_last), normFeatContext
 * slots 1..5, the LSTM h / c, and for the net at the current position its STFT
 * buffer, from which the frames its next window re-reads follow (the other
 * two nets are reset when the controller leaves them: their STFT buffers must
 * be zero).  The look-back features are recomputed on the device from the
 * voice buffer (the shared front end over the history).  NNSP_EINVAL when the
 * objects do not fit the cascade: another sequence length, a position past it,
 * an NNSPClass of another NNSP_ID, an LSTM of another width, or an STFT
 * buffer that is not the voice buffer's frames at that net's look-back.
 *
 * get_state_ref: the reverse, into the objects refs[i] point to (the pointers
 * and parameters are not changed): the controller's position and counters,
 * the voice buffer (idx_data_latest = num_frs - 1, idx_set = 0; frames older
 * than the look-backs reach, which the reference never reads again, are
 * zero), and per net the same fields; the current net's STFT buffer
 * (dataBuffer[160..479]) holds the frames its next window re-reads.  Fields
 * the reference overwrites before reading them (dataBuffer[0..159],
 * normFeatContext slot 0, FeatureClass.feature) are zero or untouched.
 * Running nnCntrlClass_exec on the result continues the stream bit-exactly. */
int nnsp_cascade_set_state_ref(nnsp_cascade *c, int first, int count, const nnsp_ref_stream *refs);
int nnsp_cascade_get_state_ref(nnsp_cascade *c, int first, int count, const nnsp_ref_stream *refs);

#ifdef __cplusplus
}
#endif
#endif
