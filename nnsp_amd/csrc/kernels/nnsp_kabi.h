/* nnsp_kabi.h -- plain-C argument blocks shared by the C host library and the
 * HIP launch layer (nnsp_kernels.hip).  No HIP or torch types. */
#ifndef NNSP_KABI_H
#define NNSP_KABI_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NN_MAX_LAYERS 10
#define NN_MAX_LSTM 10   /* LSTM layers per net (any layer may be one) */
#define NN_MAX_WIDTH 300 /* layer widths in int16: neural_nets.c's input0/1[300] (:9-10) */
#define NN_MAX_LIN 150   /* a linear layer's int32 outputs in those buffers */
#define NN_MAX_K 320     /* padded widths: 5 MFMA k-tiles of 64 */
#define NN_MAX_W 128     /* the split path's LSTM width and h/c row stride (fused path: NnRun.hs) */
#define NN_MAX_OUT 100   /* NNSPClass_exec's last layer: static int32_t output[50] (nn_speech.c:78) */
#define NN_MAX_OUT_LIN 50
#define NN_FC 0
#define NN_LSTM 1
/* compiled shapes of the split NN path (nnsp_fast.hip): FC(tanh, K 240) ->
 * LSTM(N) -> FC(relu6, N) -> FC(relu6, N) -> FC(linear, NOUT) */
#define NN_SHAPE_GENERIC 0
#define NN_SHAPE_VAD 1 /* N 28, NOUT 2  (def_nn1_vad.c) */
#define NN_SHAPE_KWS 2 /* N 64, NOUT 2  (def_nn2_kws_galaxy.c) */
#define NN_SHAPE_S2I 3 /* N 72, NOUT 41 (def_nn0_s2i.c) */
#define NN_MODE_STREAM 0 /* NNSPClass_exec over a chunk: FE features in, post-proc */
#define NN_MODE_DIRECT 1 /* NeuralNetClass_exe: 240-wide input in, raw output */

/* development probe buffer (NNSP_RECUR_CLOCKS), in longs: recur phase
 * clocks [0, 2048); fe_kernel per wave 4 each (32768 waves); proj_kernel
 * per wave 4 each (8192 waves); recur_pipe_kernel per workgroup 4 each (8192) */
#define NNSP_DCLK_FE 2048
#define NNSP_DCLK_PROJ (NNSP_DCLK_FE + 4 * 32768)
#define NNSP_DCLK_RECUR (NNSP_DCLK_PROJ + 4 * 8192)
#define NNSP_DCLK_LONGS (NNSP_DCLK_RECUR + 4 * 8192)

typedef struct {
    const int16_t *pcm;  /* [S][T][160] */
    const int16_t *tail; /* [S][320]: samples of the two frames before the chunk */
    int32_t S, T;
    const int32_t *mean, *stdR;
    int32_t norm_shift;  /* 30 - qbit_output */
    int16_t *feats;      /* [S][T][40] normalised log-Mel (context slot 5) */
    int32_t *dbg_spec;   /* optional [S*T][1024] rfft output */
    int32_t *dbg_log;    /* optional [S*T][40] log10 Mel (FeatureClass.feature) */
    /* segments (cascade): run only the streams list[0..n_list) (NULL: all S),
     * frames seg_begin[s]..T-1 (NULL: 0), input frame t read from chunk frame
     * t - lookback (negative: hist [S][H][160] frame H + t - lookback, H =
     * hist_frames >= lookback) */
    const int32_t *list;
    const int32_t *seg_begin;
    const int16_t *hist;
    int32_t n_list, lookback, hist_frames;
    int32_t seg_len;          /* > 0: a segment ends at min(T, seg_begin + seg_len) */
    /* cascade modes (FE_MODE_*): SHARED computes the log-Mel of every frame of
     * every stream once and writes it normalised with each net's mean / stdR
     * (feature_module.c:67-73) into that net's ring nring[n] [S][ring][40]
     * int16, chunk frame t at slot (abs0 + t) % ring; COLD runs only the
     * frames of a listed segment that come less than 2 frames after the net's
     * reset (fresh[s] = frames the net ran since its reset, 0..2): input frames
     * before the reset point are zero (stftModule_setDefault), the rest come
     * from pcm/hist */
    int32_t mode;
    int32_t ring, abs0;
    int16_t *nring[3];
    const int32_t *nmean[3], *nstdR[3];
    int32_t nshift[3];
    const int8_t *fresh;
    const int32_t *n_list_dev; /* non-NULL: the list length, read on the device */
    /* FE_MODE_SHARED, non-NULL: the PCM of the chunk's last hist_frames frames
     * (T >= hist_frames) is also stored to hist_out [S][hist_frames][160] --
     * the look-back history of the next chunk, written while the samples are
     * in registers anyway (replaces a separate history roll) */
    int16_t *hist_out;
    int32_t tail_stride;      /* samples between streams' tails (0: 320, a [S][320] buffer; a chunk's
                                 last two frames: T * 160) */
    int32_t port;             /* 1: the ARM_OPTIMIZED=0 build's front end (row N4): Frac15 window,
                                 fft.c's rfft, spec2pspec >> 15 */
    long long *dbg_clk;       /* development probe (NNSP_RECUR_CLOCKS): s_memtime per phase of wave 0 of
                                 workgroup 0, its first 64 frames: dbg_clk[1024 + 8 * frame + phase] */
    int32_t norm32;           /* 1: every normalisation's (feature - mean) * stdR >> shift provably fits
                                 int32 (nnsp_norm_fits32): the 32-bit clamp path */
    int32_t sched;            /* FE_MODE_SHARED: frame schedule (FE_SCHED_*, fe_kernel) */
    /* non-NULL: the workgroup's constant tables (twiddles, split, normalisation,
     * log, window, Mel) prebuilt for this mode / build by nnspk_build_fe_tables,
     * copied with 16-byte loads instead of being derived per workgroup */
    const void *tb_img;
    /* one-workgroup launches (the drop-in call): before anything else, the
     * workgroup copies in_bytes (a multiple of 16) from in_src (mapped host
     * memory) to in_dst in place of a separate host-to-device copy */
    const void *in_src;
    void *in_dst;
    int32_t in_bytes, pad4_;
} FeArgs;
#define FE_SCHED_EQUAL 0   /* equal contiguous ranges per wave */
#define FE_SCHED_GUIDED 1  /* the last-dispatched third of the waves on quarter ranges */

/* feature_module.c:67-73 in 32 bits: |log10 output| < 2^18 (|table| * 0x3796 >> 15
 * plus 15 * 0x2688), so with m = max |mean|, r = max |stdR| the 64-bit
 * (feature - mean) * stdR >> shift fits int32 when (2^18 + m) * r < 2^(31 + shift) */
static inline int nnsp_norm_fits32(const int32_t *mean, const int32_t *stdR, int n, int shift)
{
    if (shift < 0 || shift > 31) return 0;
    long long m = 0, r = 0;
    for (int i = 0; i < n; ++i) {
        const long long a = mean[i] < 0 ? -(long long)mean[i] : mean[i];
        const long long b = stdR[i] < 0 ? -(long long)stdR[i] : stdR[i];
        if (a > m) m = a;
        if (b > r) r = b;
    }
    const long long d = (1LL << 18) + m;
    if (d >= (1LL << 31)) return 0;
    return d * r < ((1LL << 31) << shift); /* d, r < 2^31: no overflow */
}

/* Cascade: where a net's segment features come from -- its ring of the shared
 * front end's normalised output, except the frames within 2 frames of the
 * net's reset, which the cold front end (FE_MODE_COLD) wrote to the net's
 * feats buffer. */
typedef struct {
    const int16_t *nring;     /* the net's normalised ring [S][ring][40]; NULL: every frame from feats */
    const int8_t *fresh;      /* [S] frames the net ran since its reset, at the segment start */
    int32_t ring, abs0, lookback, pad;
} FeatSrc;

#define FE_MODE_BATCH 0
#define FE_MODE_SHARED 1
#define FE_MODE_COLD 2

typedef struct {
    int32_t type, K, N, act;
    int32_t rows;        /* FC: N; LSTM: 16 * nrt (re-tiled, padded) */
    int32_t nrt, nkt, nkt_r;
    int32_t has_bias, bias_sh, out_sh; /* affine_Krows epilogue */
    int32_t xs_sh;       /* LSTM: shift_64b(acc, qi_rec - qi) on the input part */
    int32_t ep_off;      /* row offset into wsum / wsum_r / bias */
    int32_t acc32;       /* this layer's layer_func is the _acc32b twin (int32 wrap, shift_32b) */
    int64_t a_off, ar_off; /* byte offsets of the MFMA A fragments */
} NnLayer;

typedef struct {
    const uint8_t *A;      /* A fragments, 1 KiB per (row tile, k tile) */
    const int32_t *wsum;   /* per row: 128 * sum_k W (hi/lo split correction) */
    const int32_t *wsum_r; /* per row: 128 * sum_k W_rec */
    const int16_t *bias;   /* per row (re-tiled order for LSTM) */
    int32_t nl, acc32, nout, n_lstm;   /* acc32: every layer is an _acc32b layer */
    int32_t nn_id, thresh_prob, th_count, mixed_acc; /* mixed_acc: fc_8x16 and _acc32b layers mixed */
    int32_t lstm_n[NN_MAX_LSTM];
    NnLayer L[NN_MAX_LAYERS];
} NnImage;

typedef struct {
    int32_t S, T, mode, nl_run;
    const int16_t *feats;     /* [S][T][40] */
    const int16_t *prev5;     /* [S][5][40] */
    const int16_t *direct_in; /* [S][NN_MAX_K] (DIRECT mode) */
    int16_t *h;               /* [S][n_lstm][hs] */
    int32_t *c;               /* [S][n_lstm][hs] */
    void *post;               /* [S] post-processing state (32 B each) */
    int16_t *trig;            /* [S][T] NNSPClass_exec return value per frame */
    int32_t *logits;          /* STREAM: [S][T][nout] (NN frames only); DIRECT: [S][out_stride] */
    int32_t out_stride;
    int32_t hs;               /* h / c elements per LSTM row (>= the widest LSTM, multiple of 8) */
    /* one-workgroup launches (the drop-in call): after everything else, the
     * workgroup copies out_bytes (a multiple of 16) from out_src to out_dst
     * (mapped host memory) in place of a separate device-to-host copy; then,
     * if done is non-NULL (mapped host memory too), stores done_seq to it with
     * system-scope release: a host polling that word sees the results without
     * waiting for the stream (the kernel's end and its completion signal) */
    const void *out_src;
    void *out_dst;
    int32_t out_bytes, done_seq;
    uint32_t *done;
    /* development probe (PROBES builds, the drop-in call): s_memrealtime (100
     * MHz) at [0] the kernel's start, [1] the front end's end, [2 + i] the end
     * of layer i, [14] the post-processing's end, [15] the results copied out */
    long long *probe;         /* NNSP_PROBE_LONGS */
    /* the drop-in kernel, st_bytes > 0: the call runs out of LDS -- its staging
     * image [0, st_bytes) (in_dst's layout: the inputs copied in from mapped
     * host memory, the results copied out from there), every layer's epilogue
     * constants (st_rows rows of wsum, wsum_r, bias) and the A fragments of
     * layers st_first.. ([st_alo, st_alo + st_abytes) of NnImage.A; the rest
     * from memory).  The caller sets st_bytes; nnspk_launch_dropin the rest. */
    int32_t st_bytes, st_rows, st_first, st_abytes;
    int64_t st_alo;
    const void *st_base;      /* the device staging buffer (FeArgs.in_dst) the image mirrors */
} NnRun;
#define NNSP_PROBE_LONGS 96
#define NNSP_PROBE_BYTES (8 * NNSP_PROBE_LONGS)

/* split NN path (nnsp_fast.hip): nets with exactly one LSTM layer */
typedef struct {
    int32_t S, T, li, nstep_max;
    int32_t a_lds_bytes;
    int32_t tseq;             /* compiled shapes' recur: 16-stream tiles per workgroup, run back to back (1..4) */
    int64_t a_off;            /* byte offset in NnImage.A of the LDS-staged region */
    const int16_t *feats;     /* [S][T][40] */
    int16_t *prev5;           /* [S][5][40]; recur rolls it forward over the segment */
    void *post;               /* [S] NnPost */
    int32_t *gx;              /* [S][nstep_max][LSTM rows] exact Wx.x sums */
    int16_t *h;               /* [S][NN_MAX_W] */
    int32_t *c;               /* [S][NN_MAX_W] */
    int16_t *trig;            /* [S][T] */
    int32_t *logits;          /* [S][T][nout] or NULL */
    int16_t *out3;            /* [S][T][3] NNSPClass.outputs after each frame, or NULL */
    const int32_t *list;      /* segments, as FeArgs */
    const int32_t *seg_begin;
    int32_t n_list, seg_len;  /* seg_len as FeArgs */
    long long *dbg_clk;       /* development probe: [steps][8] s_memtime of tile 0, or NULL */
    int32_t ep_lo, ep_n;      /* epilogue rows [ep_lo, ep_lo + ep_n) staged into LDS */
    int32_t shape;            /* NN_SHAPE_* */
    int32_t ep32;             /* acc64 net whose accumulators provably fit int32: run the int32 kernels */
    /* cascade: the caller's per-frame outputs, written for every frame of the
     * segment (frames past a net switch are rewritten by the next net's
     * segment in the next round); NULL skips */
    int8_t *net_ran;          /* [S][T] NNSP_ID of this net */
    int16_t *detected;        /* [S][T] NNSPClass_exec return */
    int16_t *outputs3;        /* [S][T][3] NNSPClass.outputs */
    int32_t net_id;
    int32_t gpt;              /* proj: streams per 16-row tile (1, 2 or 4; compiled shapes) */
    int32_t fuse;             /* recur (compiled shapes, one tile per workgroup, ring features): it also runs
                                 the layers before the LSTM itself, one pipeline stage ahead -- no proj launch,
                                 no x rows through HBM (nnspk_fast_fuse_ok) */
    int32_t pad_fuse;
    int32_t *n_list_rec;      /* non-NULL: proj records the list length it ran with (stats) */
    FeatSrc fs;               /* cascade feature source (fs.nring NULL: feats) */
    const int32_t *n_list_dev; /* non-NULL: the list length, read on the device (grids sized for S) */
    /* compiled shapes: proj writes the LSTM's input x (the prefix layers'
     * int16 output, [S][nstep_max][xs] with xs = 16 * ceil(N / 16)) instead of
     * the int32 gate sums gx; recur computes Wx.x itself on MFMA */
    int16_t *xg;
} FastRun;

/* Legacy row-block primitives (affine_Krows_8x16*, rc_Krows_8x16*, rc_8x16*):
 * one thread per output row; rows come in the reference's 4-row groups
 * (remainder group last), weights interleaved as def_nn*.c store them. */
#define ROWS_AFFINE 0   /* affine_Krows: acc[] in/out, one group of <= 4 rows */
#define ROWS_RC 1       /* rc_Krows / rc_8x16: input half, shift, recurrent half + bias */
typedef struct {
    const int8_t *w, *wr;     /* input / recurrent weights */
    const int16_t *b;         /* NULL: no bias */
    const int16_t *x, *xr;    /* input / recurrent input */
    void *out;                /* activation output (int16; int32 for linear) or NULL */
    int64_t *acc;             /* ROWS_AFFINE: [rows] accumulators in/out (int32 values for acc32) */
    int32_t mode, rows, K, Kr;
    int32_t qk, qb, qi, qir;
    int32_t acc32, is_out, act;
    int32_t port;             /* 1: the ARM_OPTIMIZED=0 build (portable byte order, live align shift) */
} RowArgs;
int nnspk_launch_rows(const RowArgs *a, void *stream);
/* shift_64b / shift_32b (affine.c:565-591, affine_acc32b.c:566-592) over n values */
int nnspk_launch_shift(void *x, int shift, int n, int acc32, void *stream);

/* 32-byte device post-processing state, one per stream */
typedef struct {
    int16_t slides, trigger, argmax_last, pad0;
    int16_t counts[8];
    int16_t outputs[3], pad1;
} NnPost;

/* launch layer (nnsp_kernels.hip) */
int nnspk_launch_fe(const FeArgs *a, void *stream);
/* the front end's per-workgroup tables for the mode, build and (shared mode)
 * normalisation of *a, built once into a new device buffer *out (nnspk_free) */
int nnspk_build_fe_tables(void **out, const FeArgs *a, void *stream);
/* cascade reset: ring slots of the masked streams := each net's normalised
 * log-Mel of silence */
int nnspk_launch_nring_fill(int16_t *const nring[3], const int32_t *const nmean[3], const int32_t *const nstdR[3],
                            const int32_t nshift[3], int ring, const uint8_t *mask, int S, void *stream);
int nnspk_launch_nn(const NnImage *img, const NnRun *r, void *stream);
/* the drop-in call's front end (FE_MODE_BATCH, one stream, one frame) and NN
 * (NN_MODE_STREAM, T = 1) in one launch */
/* kin (NULL: none): a host copy of the call's in_bytes of inputs, passed in the
 * kernel arguments when they fit NNSP_DROPIN_KARG_BYTES (the LDS path only) */
#define NNSP_DROPIN_KARG_BYTES 2176
int nnspk_launch_dropin(const FeArgs *a, const NnImage *img, const NnRun *r, const void *kin, void *stream);
/* the resident drop-in worker: one workgroup that serves every later call with
 * these same arguments (r->done_seq aside) from its LDS, one request per
 * sequence number the host writes to mbox[0] (device address of mapped host
 * memory) after staging the call's inputs; seq0: the first request's, posted
 * before the launch.  It leaves when mbox[1] != 0 or after idle_ticks (100 MHz)
 * without a request.  Its stream is its own until then.
 * nnspk_dropin_worker_ok: 1 when the call runs out of LDS (the worker's form). */
int nnspk_dropin_worker_ok(const NnImage *img, const NnRun *r);
int nnspk_launch_dropin_worker(const FeArgs *a, const NnImage *img, const NnRun *r, const uint32_t *mbox,
                               uint32_t seq0, long long idle_ticks, void *stream);
int nnspk_launch_ctx_roll(int16_t *prev5, const int16_t *feats, int S, int T, const int32_t *list,
                          int n_list, const int32_t *seg_begin, int seg_len, void *stream);
int nnspk_launch_tail_roll(int16_t *tail, const int16_t *pcm, int S, int T, const int32_t *list,
                           int n_list, const int32_t *seg_begin, int seg_len, int lookback,
                           const int16_t *hist, int hist_frames, void *stream);
int nnspk_launch_synth_pcm(int16_t *out, int S, int T, unsigned long long seed, int s0, long long t0, int amp,
                           const int16_t *wavs, int n_wavs, int wav_len, int every, void *stream);
int nnspk_launch_rfft(int32_t *x, int32_t *y, int n, void *stream);
int nnspk_launch_pspec(int32_t *y, const int32_t *x, int len, int n, int shift, void *stream);
/* the ARM_OPTIMIZED=0 build's rfft(512) (y [n][514]) or, cfft_only, fft(8) (y [n][512]) */
int nnspk_launch_rfft_port(const int32_t *x, int32_t *y, int n, int cfft_only, void *stream);
/* complex.c's helpers (k_cplx) */
enum {
    NNSP_CPLX_COPY, NNSP_CPLX_AFFINE, NNSP_CPLX_INTERPROD, NNSP_CPLX_ELMTPROD, NNSP_CPLX_ADD, NNSP_CPLX_ARRY_ADD,
    NNSP_CPLX_NEG, NNSP_CPLX_SUB, NNSP_CPLX_MUL, NNSP_CPLX_INIT, NNSP_CPLX_ARRY_INIT
};
int nnspk_launch_cplx(int op, int32_t *o, int32_t *a, int32_t *b, int shift, int len, void *stream);
/* fft.c's fft(exp_nfft) / rfft(2^(exp_nfft+1)) for one vector, every size its tables serve */
int nnspk_launch_fft_dif(int32_t *x, int32_t *y, int exp_nfft, int rfft, void *stream);
int nnspk_launch_mel(const int32_t *spec, int32_t *mel, int n, void *stream);
int nnspk_launch_log10(int32_t *out, const int32_t *x, int n, int add, void *stream);
int nnspk_launch_act(int type, const int32_t *x, void *y, int n, void *stream);
int nnspk_launch_scalar(int op, const int32_t *in, int32_t *out, int n, void *stream);
int nnspk_launch_post(int nn_id, int thresh_prob, int th_count, void *post, int32_t *est,
                      void *stream);
int nnspk_launch_fe_default(int16_t *prev5, int16_t *tail, const int32_t *mean,
                            const int32_t *stdR, int norm_shift, const uint8_t *mask, int n,
                            void *stream);
int nnspk_launch_nn_default(int16_t *h, int32_t *c, void *post, int row, const uint8_t *mask,
                            int n, void *stream);
size_t nnspk_fast_lds_bytes(int which, int a_bytes, int units, int ep_rows, int shape);
int nnspk_launch_proj(const NnImage *img, const FastRun *r, int blocks, int waves, void *stream);
/* ctl non-NULL: the cascade controller runs fused into the pipelined recur
 * kernel (compiled shapes only); CascArgs is declared below */
struct CascArgs_;
int nnspk_launch_recur(const NnImage *img, const FastRun *r, int waves, const struct CascArgs_ *ctl, void *stream);
/* the compiled shape has a fused-prefix recurrence (FastRun.fuse) and its LDS
 * (all the net's weights, every epilogue row) fits two workgroups per CU;
 * int32-accumulator nets (acc32: the net or its proven-int32 acc64 form) */
int nnspk_fast_fuse_ok(int shape, int a_bytes, int ep_rows, int acc32);
int nnspk_set_lds_limit(void);
int nnspk_malloc(void **p, size_t n);
int nnspk_malloc_finegrained(void **p, size_t n); /* device memory the host writes directly, zeroed */
int nnspk_free(void *p);
int nnspk_memset(void *p, int v, size_t n, void *stream);
int nnspk_h2d(void *d, const void *h, size_t n, void *stream);
int nnspk_d2h(void *h, const void *d, size_t n, void *stream);
int nnspk_host_alloc(void **p, size_t n);   /* pinned host memory (asynchronous copies) */
/* pinned, coherent host memory that kernels read and write in place (*dev: the
 * address kernels use) */
int nnspk_host_alloc_mapped(void **p, void **dev, size_t n);
int nnspk_host_free(void *p);
int nnspk_event_sync(void *e);
int nnspk_event_done(void *e);              /* 1: the event has completed (no wait) */
int nnspk_event_spin(void *e);              /* wait for the event by polling it (no sleep / wake-up latency) */
int nnspk_d2d(void *d, const void *s, size_t n, void *stream);
int nnspk_sync(void *stream);
int nnspk_stream_spin(void *stream);  /* wait for the stream by polling it (no sleep / wake-up latency) */
int nnspk_stream_done(void *stream);  /* 1: complete, 0: work pending, < 0: minus the error code */
int nnspk_device_count(int *n);
int nnspk_set_device(int d);
int nnspk_get_device(int *d);
const char *nnspk_error_string(int e);
int nnspk_stream_create(void **s);
/* high != 0: the device's greatest stream priority (its kernels' workgroups
 * are dispatched ahead of normal-priority streams' when both wait) */
int nnspk_stream_create_prio(void **s, int high);
int nnspk_stream_destroy(void *s);
int nnspk_event_create(void **e);
int nnspk_event_create_dep(void **e); /* no timestamps: ordering between streams and host waits only */
int nnspk_event_destroy(void *e);
int nnspk_event_record(void *e, void *stream);
int nnspk_event_elapsed(float *ms, void *a, void *b);
int nnspk_stream_wait(void *stream, void *event);
int nnspk_device_info(int *cus, int *clock_khz, char *name, int name_len);


/* ---- VAD -> KWS -> S2I cascade (nnCntrlClass, evb/src/nnCntrlClass.c:152-272) ---- */
typedef struct {
    int16_t pos;              /* current_pos_seq */
    uint16_t cnt_kws;         /* cnt_timeout_kws */
    uint16_t cnt_s2i;         /* cnt_timeout_s2i */
    int16_t pad;
} CascState;

typedef struct CascArgs_ {
    int32_t S, T, len_seq, timeout_kws, timeout_s2i;
    int32_t seg_len;          /* frames per round and stream (0: to the chunk end) */
    int16_t seq[8];           /* net id per sequence position (0 s2i, 1 vad, 2 kws) */
    CascState *st;            /* [S] */
    int32_t *seg_begin;       /* [S] first frame of this round's segment (T: done) */
    const int16_t *trig[3];   /* per net id: [S][T] triggers of the round's segments */
    const int16_t *feats[3];  /* per net id: [S][T][40] */
    int16_t *prev5[3];        /* per net id: [S][5][40] */
    int16_t *h[3];            /* per net id: [S][NN_MAX_W] LSTM state (one LSTM layer) */
    int32_t *c[3];
    void *post[3];            /* per net id: [S] NnPost */
    const int16_t *prev_default[3]; /* per net id: [40] FeatureClass_setDefault context value */
    int32_t *list[3];         /* per net id: next round's streams */
    int32_t *cold_list[3];    /* per net id: those of them within 2 frames of the net's reset */
    int32_t *counts;          /* [6] next round's list lengths (appended to): lists, cold lists */
    int32_t *counts_clear;    /* [6] zeroed by casc_control: the round after next appends there */
    int32_t *last_round;      /* atomicMax'ed with round + 1 when a stream is listed for it */
    int32_t round;            /* index of the round casc_control closes */
    unsigned long long *frames; /* [3] frames scheduled per net id (speculation included) */
    int8_t *net_ran;          /* [S][T] or NULL */
    int16_t *detected;        /* [S][T] or NULL */
    int16_t *outputs3;        /* [S][T][3] or NULL */
    int8_t *fresh;            /* [S] frames the current net ran since its reset (0..2) */
    FeatSrc fs[3];            /* per net id: segment feature source (slot 5 kept at a reset) */
    int32_t *cuts;            /* segments cut by a net switch this chunk (window heuristic), or NULL */
    int32_t seq_bits;         /* seq[k] in bits 2k..2k+1 (per-lane lookups without a memory load) */
    int32_t pad_;
} CascArgs;

int nnspk_launch_casc_begin(const CascArgs *a, void *stream);
int nnspk_launch_casc_control(const CascArgs *a, void *stream);
int nnspk_launch_casc_reset(CascState *st, int16_t *hist, int hist_frames, int16_t *stail, int8_t *fresh,
                            const uint8_t *mask, int S, void *stream);
int nnspk_launch_hist_roll(int16_t *dst, const int16_t *src, const int16_t *pcm, int S, int T,
                           int hist_frames, void *stream);

/* ---- per-stream state export / import (nnsp_batch_get_state, nnsp_cascade_get_state) ----
 * A stream's blob is a list of segments.  Segment k of stream s is `rows` rows
 * of `row_bytes` bytes: row r lies at base + s * stride + ((row0 + r) % wrap) *
 * row_pitch on the device (wrap: a ring's slot count; 1 for plain arrays) and
 * at off + r * row_bytes in the blob.  The kernel gathers the blobs of streams
 * first .. first + count - 1 into blob [count][per] (to_blob) or scatters them
 * back. */
#define NNSP_STATE_SEGS 24
typedef struct {
    unsigned long long base, stride, row_pitch;
    uint32_t rows, row_bytes, row0, wrap, off, pad_;
} StateSeg;
typedef struct {
    StateSeg seg[NNSP_STATE_SEGS];
    int32_t nseg, first, count, to_blob;
    unsigned long long per;
} StateCopy;
int nnspk_launch_state_copy(const StateCopy *sc, void *blob, void *stream);

#ifdef __cplusplus
}
#endif
#endif
