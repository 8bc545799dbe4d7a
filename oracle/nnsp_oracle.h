/*
 * nnsp_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * Scalar CPU restatement of the ns-nnsp per-frame hot path (ARM_OPTIMIZED=1
 * build) used as the parity checker for the MI355X implementation and as the
 * CPU baseline ("port") in bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product library never does.
 *
 * Parity status (details in DESIGN.md "Oracle"):
 *   - constant tables: pinned byte-exact against the reference source tables
 *     and the CMSIS-DSP data sections (tests/test_tables.py);
 *   - post-FFT front end, activations, post-processing, reset logic: pinned
 *     against reference C files compiled here from their own sources
 *     (oracle/_ref -> tests/golden/ref_stages.npz, tests/test_oracle_pinned.py);
 *   - weight layout: pinned against python/nnsp_pack/c_weight_man.py;
 *   - affine / rc / LSTM / NeuralNetClass_exe: pinned against the
 *     reference's own portable NN build (affine.c, affine_acc32b.c, lstm.c,
 *     neural_nets.c compiled with ARM_OPTIMIZED=0 -> tests/golden/ref_nn.npz)
 *     on re-packed weights, including the reference's three nets; that build
 *     differs from the shipped one only in the byte walk (pinned by
 *     layout.npz) and the live align shift (or_net.portable = 1 reproduces
 *     it; the shipped build's dead shift is trap T1);
 *   - CMSIS arm_rfft_q31 (binary-only third-party code): restated, "parity
 *     unpinned" beyond its tables and a float-DFT check.
 */
#ifndef NNSP_ORACLE_H
#define NNSP_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_MAX_LAYERS 10
#define OR_MAX_LSTM 10   /* any layer of a NeuralNetClass may be an LSTM */
#define OR_MAX_WIDTH 304 /* >= neural_nets.c's 300-element activation buffers (:9-10) */

enum { OR_RELU6 = 0, OR_TANH = 1, OR_SIGMOID = 2, OR_LINEAR = 3 };
enum { OR_FC = 0, OR_LSTM = 1 };

/* Net description: the data a NeuralNetClass carries (neural_nets.h:15-32),
 * with the layer/activation function pointers replaced by enums. */
typedef struct {
    int32_t nl;
    int32_t size[OR_MAX_LAYERS + 1];
    int32_t type[OR_MAX_LAYERS];
    int32_t qk[OR_MAX_LAYERS];
    int32_t qi[OR_MAX_LAYERS];
    int32_t qb[OR_MAX_LAYERS];
    int32_t act[OR_MAX_LAYERS];
    int32_t acc32; /* 1: *_acc32b layer functions (DEF_ACC32BIT_OPT) */
    const int8_t *W[OR_MAX_LAYERS];
    const int8_t *Wr[OR_MAX_LAYERS];
    const int16_t *B[OR_MAX_LAYERS];
    int32_t portable; /* 1: the ARM_OPTIMIZED=0 build's live align shift (affine.c:311-313), 0: shipped (T1) */
    int32_t acc32_layer[OR_MAX_LAYERS]; /* per layer: its layer_func is the _acc32b twin (ORed with acc32) */
} or_net;

/* Per-stream state of one NNSPClass + FeatureClass + LSTM h/c. */
typedef struct {
    int16_t buf[480];  /* stftModule.dataBuffer[0..479] */
    int16_t ctx[240];  /* FeatureClass.normFeatContext[0..239], oldest first */
    int16_t h[OR_MAX_LSTM][OR_MAX_WIDTH];
    int32_t c[OR_MAX_LSTM][OR_MAX_WIDTH];
    int16_t slides, trigger, argmax_last, pad0;
    int16_t counts[8];
    int16_t outputs[3];
    int16_t pad1;
} or_stream;

/* Post-processing parameters (pointed to by NNSPClass.pt_thresh_prob /
 * pt_th_count_trigger). */
typedef struct {
    int32_t nn_id; /* 0 s2i, 1 vad, 2 kws */
    int32_t thresh_prob;
    int32_t th_count;
    int32_t qbit_out; /* FeatureClass.qbit_output = net qbit_input[0] */
    const int32_t *mean;
    const int32_t *stdR;
    int32_t fe_portable; /* 1: the ARM_OPTIMIZED=0 build's FFT front end (row N4) */
} or_cfg;

/* front end stages */
void or_rfft512(int32_t *x, int32_t *y); /* x: 512 q31 (clobbered); y: 1024 q31 */
void or_rfft512_portable(const int32_t *x, int32_t *y); /* ARM_OPTIMIZED=0 rfft: x 512 Frac15; y 257 complex */
void or_spec2pspec(int32_t *y, const int32_t *x, int n);
void or_mel(const int32_t *pspec, int32_t *mel);
int32_t or_log10(int32_t x);
void or_fe_reset(or_stream *st, const or_cfg *cfg);
void or_fe_exec(or_stream *st, const or_cfg *cfg, const int16_t *pcm160);

/* activations (type = OR_*); y is int16 except OR_LINEAR (int32) */
void or_act(int32_t type, const int32_t *x, void *y, int32_t n);
/* row-block primitives as the legacy API exposes them (test entry points):
 * affine_Krows_8x16(_acc32b) on R <= 4 rows with accumulators in/out (int32
 * values for acc32; b NULL: no bias); rc_8x16(_acc32b) on a whole layer of N
 * rows in 4-row groups; shift_64b / shift_32b */
void or_affine_krows(int32_t R, const int8_t *w, const int16_t *b, const int16_t *x, int32_t K, int32_t qk,
                     int32_t qb, int32_t qi, int64_t *acc, int32_t acc32, int32_t is_out, int32_t act, void *out);
void or_rc_layer(int32_t N, const int8_t *w, const int8_t *wr, const int16_t *b, const int16_t *x,
                 const int16_t *h, int32_t K, int32_t Kr, int32_t qk, int32_t qb, int32_t qi, int32_t qir,
                 int32_t act, int32_t acc32, void *out);
void or_shift(int64_t *a, int32_t sh, int32_t n, int32_t acc32);
/* fc_8x16(_acc32b) / lstm_8x16(_acc32b) on a whole layer (natural order of the
 * interleaved weight stream; h / c updated in place).  portable: see or_net. */
void or_fc(int32_t N, const int8_t *w, const int16_t *b, const int16_t *x, int32_t K, int32_t qk, int32_t qb,
           int32_t qi, int32_t act, int32_t acc32, int32_t portable, void *out);
void or_lstm(int32_t N, const int8_t *w, const int8_t *wr, const int16_t *b, const int16_t *x, int16_t *h,
             int32_t *c, int32_t K, int32_t qk, int32_t qb, int32_t qi, int32_t qir, int32_t acc32,
             int32_t portable, int16_t *out);

/* NN */
void or_nn_reset(const or_net *net, or_stream *st);
void or_net_forward(const or_net *net, or_stream *st, const int16_t *in, int32_t *out,
                    int32_t n_layers);

/* post-processing */
int32_t or_ceiling(int32_t x);
int32_t or_pwr2(int32_t x);
void or_binary_post(or_stream *st, const or_cfg *cfg, int32_t *est);
void or_s2i_post(or_stream *st, const or_cfg *cfg, int32_t *est);

/* NNSPClass */
void or_nnsp_reset(const or_net *net, or_stream *st, const or_cfg *cfg);
int16_t or_nnsp_exec(const or_net *net, or_stream *st, const or_cfg *cfg,
                     const int16_t *pcm160, int32_t *logits /* may be NULL */,
                     int32_t *ran_nn /* may be NULL */);

/* S streams x T frames, frame-major per stream (stream-sequential).
 * pcm [S][T][160]; trig [S][T]; logits [S][T][nout] (NULL ok; rows of frames
 * without an NN step are left untouched); feat [S][T][40] = ctx slot 5 after
 * each frame (NULL ok). */
void or_run_streams(const or_net *net, const or_cfg *cfg, or_stream *st, int32_t S,
                    int32_t T, const int16_t *pcm, int16_t *trig, int32_t *logits,
                    int16_t *feat);

/* VAD -> KWS -> S2I cascade (evb/src/nnCntrlClass.c:152-272), one stream. */
typedef struct {
    int16_t ring[100 * 160];
    int16_t idx_set, idx_latest;
    int16_t pos_seq, pad;
    uint16_t cnt_timeout_kws, cnt_timeout_s2i;
    or_stream nnsp[3]; /* indexed by nn id: 0 s2i, 1 vad, 2 kws */
} or_cascade;

typedef struct {
    const or_net *net[3];
    or_cfg cfg[3];
    int32_t seq[3];
    int32_t len_seq;
    int32_t lookback_kws, lookback_s2i;
    int32_t timeout_kws, timeout_s2i;
} or_cascade_cfg;

void or_cascade_reset(or_cascade *c, const or_cascade_cfg *cfg);
/* returns the id of the net that ran this frame; *detected = its trigger */
int32_t or_cascade_exec(or_cascade *c, const or_cascade_cfg *cfg, const int16_t *pcm160,
                        int16_t *detected, int16_t *out3);
void or_run_cascade(const or_cascade_cfg *cfg, or_cascade *c, int32_t S, int32_t T,
                    const int16_t *pcm, int8_t *net_ran, int16_t *detected, int16_t *outputs3);

int32_t or_sizeof_stream(void);
int32_t or_sizeof_cascade(void);

#ifdef __cplusplus
}
#endif
#endif
