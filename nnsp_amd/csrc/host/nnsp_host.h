/* nnsp_host.h -- internal declarations of the C host library. */
#ifndef NNSP_HOST_H
#define NNSP_HOST_H
#include <stddef.h>
#include <stdint.h>

#include "../../../include/nnsp_api.h"
#include "../kernels/nnsp_kabi.h"
#include "../../../include/nnsp_batch.h"

/* error codes: NNSP_EINVAL / NNSP_EUNSUPPORTED / NNSP_ENOMEM (include/nnsp_batch.h) */

/* One layer as the engine sees it (what a NeuralNetClass row describes). */
typedef struct {
    int type;                 /* NN_FC / NN_LSTM */
    int K, N;                 /* input width, output width (LSTM: units) */
    int act;                  /* device activation enum (FC only) */
    int acc32;
    int qk, qb, qi, qir;
    const int8_t *W, *Wr;     /* interleaved byte streams (def_nn*.c layout) */
    const int16_t *B;         /* NULL: no bias */
    int portable;             /* the ARM_OPTIMIZED=0 build (row N4): W / Wr in the portable byte order
                                 (per 4-row block, per column pair, per row; affine.c:261-346) and the
                                 live align shift (affine.c:311-313) */
} nnsp_layer_desc;

typedef struct {
    NnImage img;              /* device pointers valid after upload */
    uint8_t *A;
    int32_t *wsum, *wsum_r;
    int16_t *bias;
    size_t a_bytes;
    int rows_total;
    void *dA, *dwsum, *dwsum_r, *dbias;
} nnsp_image;

int nnsp_describe_net(const NeuralNetClass *net, nnsp_layer_desc *L, int *nl, int *out_linear);
int nnsp_image_build(nnsp_image *im, const nnsp_layer_desc *L, int nl, int nn_id,
                     int thresh_prob, int th_count, int direct);
int nnsp_image_upload(nnsp_image *im, void *stream);
void nnsp_image_free(nnsp_image *im);

/* activation function pointer -> device enum (-1 unknown) */
int nnsp_act_of(void *(*fn)(void *, int32_t *, int));

/* the batch engine's internals, shared with the cascade (nnsp_cascade.c) */
struct nnsp_batch {
    int S, Tmax, nout, out_linear, norm_shift;
    int nn_id;                        /* NNSP_ID given at create (post-processing kind) */
    int port;                         /* 1: the ARM_OPTIMIZED=0 build (row N4), nnsp_batch_create_ex */
    int norm32;                       /* normalisation fits int32 (nnsp_norm_fits32) */
    nnsp_image im;
    void *stream;
    void *ev[3];
    int32_t *d_mean, *d_stdR;
    int16_t *d_tail, *d_prev5, *d_h;
    int32_t *d_c;
    NnPost *d_post;
    int16_t *d_feats, *d_pcm, *d_trig;
    int32_t *d_logits;
    uint8_t *d_mask;
    int last_T;
    /* split NN path (one LSTM layer) */
    int fast, li, nstep_max, rec_waves, proj_blocks, proj_waves;
    int fuse;                         /* the cascade's whole-segment VAD rounds run the prefix layer inside recur
                                         (FastRun.fuse; NNSP_FUSE_PREFIX) */
    int ep_proj, ep_rec_lo, ep_rec_n; /* epilogue rows staged into LDS by proj / recur */
    int shape;                        /* NN_SHAPE_* compiled split-path shape */
    int ep32;                         /* acc64 net that provably fits int32 accumulators */
    int hs;                           /* h / c elements per LSTM row of the state (NN_MAX_W or wider) */
    int32_t *d_gx;                    /* generic shape: proj -> recur exact Wx.x sums */
    int16_t *d_xg;                    /* compiled shapes: proj -> recur LSTM inputs x */
    long long rec_a_off;              /* first byte of the image recur stages into LDS */
    long long *d_clk; /* NNSP_RECUR_CLOCKS development probe */
    void *d_fetab;    /* the front end's per-workgroup tables, prebuilt (nnspk_build_fe_tables) */
};

/* One segment launch of a batch: the streams list[0..n_list) (NULL: all),
 * frames seg_begin[s]..T-1 (NULL: 0), input frame t = chunk frame t - lookback
 * (earlier frames from hist [S][hist_frames][160]); out3 [S][T][3] optional. */
typedef struct {
    const int32_t *list;
    const int32_t *seg_begin;
    const int16_t *hist;
    int16_t *out3;
    int n_list, lookback, hist_frames;
    int seg_len;              /* > 0: segments end at min(T, seg_begin + seg_len) */
    const int32_t *n_list_dev; /* non-NULL: list length on the device (overrides n_list) */
    int32_t *n_list_rec;       /* non-NULL: the list length proj ran with is recorded there */
    FeatSrc fs;                /* cascade feature source (fs.nring NULL: the batch's feats) */
    int8_t *net_ran;           /* cascade: the caller's per-frame outputs (NULL skips) */
    int16_t *detected, *outputs3;
    int net_id;
    const CascArgs *ctl;       /* cascade: controller fused into recur (NULL: none) */
    void *proj_done;           /* non-NULL: recorded on the stream once the prefix FC layers are done
                                  (split path: between proj and recur; fused kernel: after it) */
    void *recur_wait[2];       /* split path: events the recurrence waits for after proj (NULL: none) */
    int round;                 /* cascade round (0: the chunk's first) */
} nnsp_segment;

int nnsp_batch_run(nnsp_batch *b, const int16_t *pcm, int T, int16_t *trig, int32_t *logits,
                   const nnsp_segment *seg, void *stream, int timed);
/* the NN half of a segment run (features already in d_feats): proj + recur
 * (or the fused kernel) and the feature-context roll */
int nnsp_batch_run_nn(nnsp_batch *b, int T, int16_t *trig, int32_t *logits, const nnsp_segment *seg,
                      void *stream);

/* per-stream state blobs (StateCopy): the batch's segments appended at blob
 * offset off (returns the count appended, sets *end past them), and the
 * gather / scatter of streams first .. first + count - 1 through a device
 * staging buffer to / from host [count][sc->per] */
int nnsp_batch_state_segs(const nnsp_batch *b, StateSeg *seg, size_t off, size_t *end);
int nnsp_state_xfer(StateCopy *sc, void *host, void *stream);

void nnsp_set_error(const char *fmt, ...);
const char *nnsp_last_error(void);

#endif
