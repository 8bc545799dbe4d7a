/*
 * nnsp_batch.c -- the batched multi-stream engine (include/nnsp_batch.h).
 *
 * Device state per stream (everything NNSPClass_exec carries between frames):
 *   tail  [320] int16   stftModule.dataBuffer[160..479] (spectrogram_module.c:103-108)
 *   prev5 [5][40] int16 normFeatContext slots 1..5     (feature_module.c:54-57)
 *   h/c   [n_lstm][128]  LSTM state                     (def_nn*.c pt_hstate/pt_cstate)
 *   post  32 B           slides, trigger, counts, outputs, argmax_last (nn_speech.h:12-25)
 * A chunk of T frames runs as: fe_kernel (all S*T frames in parallel) ->
 * nn_kernel (per 16-stream tile, the chunk's NN steps in order) -> roll of the
 * feature context and the PCM tail.
 */
#include <stdlib.h>
#include <string.h>

#include "nnsp_host.h"

#define LDS_MAX (160 * 1024)

/* Which compiled shape of the split kernels fits this net (nnsp_fast.hip):
 * FC(tanh, 240 -> N) -> LSTM(N) -> FC(relu6, N) -> FC(relu6, N) -> FC(linear). */
static int net_shape(const NnImage *g)
{
    static const int known[3][3] = {{NN_SHAPE_VAD, 28, 2}, {NN_SHAPE_KWS, 64, 2}, {NN_SHAPE_S2I, 72, 41}};
    if (g->nl != 5 || g->n_lstm != 1) return NN_SHAPE_GENERIC;
    const NnLayer *L = g->L;
    if (L[0].type != NN_FC || L[1].type != NN_LSTM || L[2].type != NN_FC || L[3].type != NN_FC ||
        L[4].type != NN_FC)
        return NN_SHAPE_GENERIC;
    if (L[0].K != 240 || L[0].act != 1 /* tanh */ || L[2].act != 0 /* relu6 */ || L[3].act != 0 ||
        L[4].act != 3 /* linear */)
        return NN_SHAPE_GENERIC;
    /* the compiled recur adds the LSTM's input and recurrent halves in one
     * accumulator: rc_Krows' shift of the input half must be 0 (qi_rec = qi) */
    if (L[1].xs_sh != 0) return NN_SHAPE_GENERIC;
    const int N = L[1].N;
    if (L[0].N != N || L[1].K != N || L[2].K != N || L[2].N != N || L[3].K != N || L[3].N != N || L[4].K != N)
        return NN_SHAPE_GENERIC;
    for (int i = 0; i < 3; ++i)
        if (N == known[i][1] && L[4].N == known[i][2])
            /* the 2-output shapes compile binary post-processing only: an s2i
             * post-processing (nn_id 0) on them takes the generic kernels */
            return known[i][2] < 41 && g->nn_id == 0 ? NN_SHAPE_GENERIC : known[i][0];
    return NN_SHAPE_GENERIC;
}

/* An acc64 net runs on the int32-accumulator kernels when every accumulator
 * provably stays inside int32: |sum_k W x| <= K * max|W| * 2^15 per half
 * (activations are int16) plus the aligned bias.  Without overflow the two
 * builds compute the same values -- shift_64b's clamp to int32
 * (affine.c:242-249) never binds and shift_32b (affine_acc32b.c:243-250)
 * never wraps -- provided no left (saturating) shift is involved. */
static int fits_int32(const nnsp_batch *b, const nnsp_layer_desc *L, int nl)
{
    const NnImage *g = &b->im.img;
    const long long LIM = 2147483647LL;
    for (int i = 0; i < nl; ++i) {
        const NnLayer *Ly = &g->L[i];
        if (Ly->out_sh > 0 || Ly->xs_sh != 0) return 0;
        const int lstm = L[i].type == NN_LSTM;
        const int rows = lstm ? 4 * L[i].N : L[i].N;
        long long wmax = 0, rmax = 0, bmax = 0;
        for (size_t k = 0; k < (size_t)rows * (size_t)L[i].K; ++k) {
            const long long v = L[i].W[k] < 0 ? -(long long)L[i].W[k] : L[i].W[k];
            if (v > wmax) wmax = v;
        }
        if (lstm && L[i].Wr)
            for (size_t k = 0; k < (size_t)rows * (size_t)L[i].N; ++k) {
                const long long v = L[i].Wr[k] < 0 ? -(long long)L[i].Wr[k] : L[i].Wr[k];
                if (v > rmax) rmax = v;
            }
        if (L[i].B)
            for (int r = 0; r < rows; ++r) {
                const long long v = L[i].B[r] < 0 ? -(long long)L[i].B[r] : L[i].B[r];
                if (v > bmax) bmax = v;
            }
        long long bound = (long long)L[i].K * wmax * 32768 + (lstm ? (long long)L[i].N * rmax * 32768 : 0);
        if (Ly->has_bias) bound += Ly->bias_sh >= 0 ? (Ly->bias_sh < 32 ? bmax << Ly->bias_sh : LIM) : bmax;
        if (bound >= LIM) return 0;
    }
    return 1;
}

/* Use the split proj/recur kernels when the net has exactly one LSTM layer,
 * every other layer is FC and the staged weights fit in LDS. */
static void plan_fast(nnsp_batch *b)
{
    const NnImage *g = &b->im.img;
    b->fast = 0;
    if (getenv("NNSP_FUSED_NN")) return;
    /* the split kernels: one accumulator width (template), one LSTM of width
     * <= NN_MAX_W (its state rows), prefix layers of <= 4 k-tiles and <= 256
     * rows, suffix layers <= 128 wide (their LDS rows); anything else the
     * reference runs goes to the fused nn_kernel */
    if (g->n_lstm != 1 || g->mixed_acc) return;
    int li = -1;
    for (int i = 0; i < g->nl; ++i)
        if (g->L[i].type == NN_LSTM) li = i;
    if (g->L[li].N > NN_MAX_W || g->L[li].K > 256) return;
    for (int i = 0; i < li; ++i)
        if (g->L[i].N > 256 || g->L[i].K > 256) return;
    for (int i = li + 1; i < g->nl; ++i)
        if (g->L[i].N > 128 || g->L[i].K > 128) return;
    const int shape = getenv("NNSP_GENERIC_SHAPE") ? NN_SHAPE_GENERIC : net_shape(g);
    /* compiled shapes: proj runs the layers before the LSTM and hands the
     * LSTM's input x to recur, which stages the LSTM's input AND recurrent
     * fragments; generic: proj also runs the input half (exact int32 gx) */
    const int xmode = shape != NN_SHAPE_GENERIC;
    const size_t rec_lo = xmode ? (size_t)g->L[li].a_off : (size_t)g->L[li].ar_off;
    const int a_proj = xmode ? (int)g->L[li].a_off : (int)g->L[li].ar_off;
    const int a_rec = (int)(b->im.a_bytes - rec_lo);
    b->rec_a_off = (long long)rec_lo;
    /* epilogue rows: proj covers layers 0..li (xmode: 0..li-1), recur li..nl-1 */
    b->ep_proj = g->L[li].ep_off + (xmode ? 0 : 16 * g->L[li].nrt);
    b->ep_rec_lo = g->L[li].ep_off;
    b->ep_rec_n = b->im.rows_total - g->L[li].ep_off;
    /* proj workgroups of 4 or 8 waves (they share the staged weights), whichever
     * keeps more waves per CU resident (LDS-bound) */
    int wpb = 4, per_cu = 0;
    for (int w = 4; w <= 8; w += 4) {
        const size_t lds = nnspk_fast_lds_bytes(0, a_proj, w, b->ep_proj, shape);
        int fit = lds <= LDS_MAX ? (int)(LDS_MAX / lds) : 0;
        if (fit * w > 32) fit = 32 / w;
        if (fit * w > per_cu * wpb) {
            per_cu = fit;
            wpb = w;
        }
    }
    if (per_cu < 1) return;
    b->proj_waves = wpb;
    if (nnspk_fast_lds_bytes(1, a_rec, 1, b->ep_rec_n, shape) > LDS_MAX) return;
    /* tiles per 4-wave group in one workgroup: 2 once there are >= 2 tiles per CU */
    const int tiles = (b->S + 15) / 16;
    b->rec_waves = (tiles >= 512 && nnspk_fast_lds_bytes(1, a_rec, 2, b->ep_rec_n, shape) <= LDS_MAX) ? 2 : 1;
    b->li = li;
    b->shape = shape;
    b->nstep_max = (b->Tmax + 1) / 2;
    /* proj: a persistent grid of as many 4-wave workgroups as fit on the
     * device at once (LDS-bound, at most 8 per CU); (round 3: 2x / 4x that
     * grid, for finer balance as in the front end: cascade 1.008 / 0.998 vs
     * 1.010 G, VAD 1.219 / 1.184 vs 1.194 G -- no gain) */
    int cus = 256, clk = 0;
    char arch[64];
    if (nnspk_device_info(&cus, &clk, arch, (int)sizeof arch) || cus <= 0) cus = 256;
    const long long ptiles = (long long)b->S * ((b->nstep_max + 15) / 16);
    long long blocks = (ptiles + wpb - 1) / wpb;
    const long long cap = (long long)cus * per_cu;
    b->proj_blocks = (int)(blocks < cap ? blocks : cap);
    b->fast = 1;
}

/* NNSP_RECUR_CLOCKS probe buffer (layout: nnsp_kabi.h NNSP_DCLK_*) */
#define DCLK_LONGS NNSP_DCLK_LONGS

#define TRY(x)                 \
    do {                       \
        int _e = (x);          \
        if (_e) return _e;     \
    } while (0)

int nnsp_device_count(int *n) { return nnspk_device_count(n); }
int nnsp_set_device(int dev) { return nnspk_set_device(dev); }
int nnsp_device_info(int *cu, int *clk, char *arch, int len) { return nnspk_device_info(cu, clk, arch, len); }

const char *nnsp_strerror(int code)
{
    if (code == 0) return "ok";
    if (code < 0) return nnsp_last_error()[0] ? nnsp_last_error() : "invalid argument";
    return nnspk_error_string(code);
}

int nnsp_batch_create(nnsp_batch **out, const NeuralNetClass *net, int nn_id, const int32_t *mean,
                      const int32_t *stdR, int16_t thresh_prob, int16_t th_count, int n_streams,
                      int max_frames)
{
    return nnsp_batch_create_ex(out, net, nn_id, mean, stdR, thresh_prob, th_count, n_streams, max_frames, 1);
}

int nnsp_batch_create_ex(nnsp_batch **out, const NeuralNetClass *net, int nn_id, const int32_t *mean,
                         const int32_t *stdR, int16_t thresh_prob, int16_t th_count, int n_streams,
                         int max_frames, int arm_optimized)
{
    *out = NULL;
    if (arm_optimized != 0 && arm_optimized != 1) {
        nnsp_set_error("nnsp_batch_create_ex: arm_optimized must be 0 or 1");
        return NNSP_EINVAL;
    }
    if (!net || !mean || !stdR || n_streams <= 0 || max_frames <= 0) {
        nnsp_set_error("nnsp_batch_create: bad argument");
        return NNSP_EINVAL;
    }
    if ((long long)n_streams * max_frames >= (1LL << 31) / 2) {
        nnsp_set_error("n_streams * max_frames must stay below 2^30");
        return NNSP_EINVAL;
    }
    if (net->size_layer[0] != NUM_FEATURE_CONTEXT * DIMEMSION_FEATURE) {
        nnsp_set_error("net input width %d != 240 (6 x 40 context)", net->size_layer[0]);
        return NNSP_EINVAL;
    }
    nnsp_layer_desc L[NN_MAX_LAYERS];
    int nl = 0, out_linear = 0;
    TRY(nnsp_describe_net(net, L, &nl, &out_linear));
    for (int i = 0; i < nl; ++i) L[i].portable = !arm_optimized;
    nnsp_batch *b = (nnsp_batch *)calloc(1, sizeof *b);
    if (!b) return NNSP_ENOMEM;
    *out = b;
    b->S = n_streams;
    b->Tmax = max_frames;
    b->nn_id = nn_id;
    b->port = !arm_optimized;
    b->out_linear = out_linear;
    b->norm_shift = 30 - net->qbit_input[0]; /* FeatureClass qbit_output, nn_speech.c:40-44 */
    b->norm32 = nnsp_norm_fits32(mean, stdR, 40, b->norm_shift);
    int e = nnsp_image_build(&b->im, L, nl, nn_id, thresh_prob, th_count, 0);
    if (e) goto fail;
    b->nout = b->im.img.nout;
    if ((e = nnspk_stream_create(&b->stream))) goto fail;
    for (int i = 0; i < 3; ++i)
        if ((e = nnspk_event_create(&b->ev[i]))) goto fail;
    if ((e = nnsp_image_upload(&b->im, b->stream))) goto fail;
    const size_t S = (size_t)n_streams, T = (size_t)max_frames;
    const int nls = b->im.img.n_lstm ? b->im.img.n_lstm : 1;
    /* h / c row stride: NN_MAX_W, or the widest LSTM rounded up to 8 */
    b->hs = NN_MAX_W;
    for (int i = 0; i < b->im.img.n_lstm; ++i)
        if (b->im.img.lstm_n[i] > b->hs) b->hs = (b->im.img.lstm_n[i] + 7) / 8 * 8;
    if ((e = nnspk_malloc((void **)&b->d_mean, 40 * 4))) goto fail;
    if ((e = nnspk_malloc((void **)&b->d_stdR, 40 * 4))) goto fail;
    if ((e = nnspk_malloc((void **)&b->d_tail, S * 320 * 2))) goto fail;
    if ((e = nnspk_malloc((void **)&b->d_prev5, S * 200 * 2))) goto fail;
    if ((e = nnspk_malloc((void **)&b->d_h, S * nls * (size_t)b->hs * 2))) goto fail;
    if ((e = nnspk_malloc((void **)&b->d_c, S * nls * (size_t)b->hs * 4))) goto fail;
    if ((e = nnspk_malloc((void **)&b->d_post, S * sizeof(NnPost)))) goto fail;
    if ((e = nnspk_malloc((void **)&b->d_feats, S * T * 40 * 2))) goto fail;
    if ((e = nnspk_malloc((void **)&b->d_mask, S))) goto fail;
    plan_fast(b);
    b->ep32 = !b->im.img.acc32 && !b->im.img.mixed_acc && !getenv("NNSP_NO_EP32") && fits_int32(b, L, nl);
    {   /* the fused prefix (VAD): recur also runs the layer before the LSTM,
         * one pipeline stage ahead, for segments of whole chunks on the
         * cascade's ring (nnsp_batch_run_nn) */
        const char *fe = getenv("NNSP_FUSE_PREFIX");
        b->fuse = b->fast && (fe ? atoi(fe) != 0 : 0) &&
                  nnspk_fast_fuse_ok(b->shape, (int)b->im.a_bytes, b->im.rows_total, b->im.img.acc32 || b->ep32);
        /* 2 (tests): a VAD net that cannot fuse is an error rather than a silent fallback */
        if (fe && atoi(fe) == 2 && b->fast && b->shape == NN_SHAPE_VAD && !b->fuse) {
            nnsp_set_error("nnsp_batch_create: NNSP_FUSE_PREFIX=2 and the net cannot run the fused prefix");
            e = NNSP_EUNSUPPORTED;
            goto fail;
        }
    }
    if (b->fast) {
        if ((e = nnspk_set_lds_limit())) goto fail;
        if (b->shape != NN_SHAPE_GENERIC) { /* x rows: int16, 16 * ceil(N / 16) per (stream, step) */
            const size_t xs = (size_t)(b->im.img.L[b->li].N + 15) / 16 * 16;
            if ((e = nnspk_malloc((void **)&b->d_xg, S * (size_t)b->nstep_max * xs * 2))) goto fail;
        } else {
            const size_t rows = (size_t)b->im.img.L[b->li].rows;
            if ((e = nnspk_malloc((void **)&b->d_gx, S * (size_t)b->nstep_max * rows * 4))) goto fail;
        }
        if (getenv("NNSP_RECUR_CLOCKS")) { /* development probe of recur_kernel phases */
            if ((e = nnspk_malloc((void **)&b->d_clk, DCLK_LONGS * 8))) goto fail;
            if ((e = nnspk_memset(b->d_clk, 0, DCLK_LONGS * 8, b->stream))) goto fail;
        }
    }
    if ((e = nnspk_h2d(b->d_mean, mean, 40 * 4, b->stream))) goto fail;
    if ((e = nnspk_h2d(b->d_stdR, stdR, 40 * 4, b->stream))) goto fail;
    if ((e = nnspk_memset(b->d_prev5, 0, S * 200 * 2, b->stream))) goto fail;
    if ((e = nnspk_memset(b->d_post, 0, S * sizeof(NnPost), b->stream))) goto fail;
    {
        FeArgs ta;
        memset(&ta, 0, sizeof ta);
        ta.mode = FE_MODE_BATCH;
        ta.port = b->port;
        if ((e = nnspk_build_fe_tables(&b->d_fetab, &ta, b->stream))) goto fail;
    }
    if ((e = nnsp_batch_reset(b, NULL))) goto fail;
    return 0;
fail:
    nnsp_batch_destroy(b);
    *out = NULL;
    return e;
}

void nnsp_batch_destroy(nnsp_batch *b)
{
    if (!b) return;
    if (b->stream) nnspk_sync(b->stream);
    nnsp_image_free(&b->im);
    void *bufs[] = {b->d_mean, b->d_stdR, b->d_tail, b->d_prev5, b->d_h, b->d_c, b->d_post,
                    b->d_feats, b->d_pcm, b->d_trig, b->d_logits, b->d_mask, b->d_gx, b->d_xg, b->d_clk,
                    b->d_fetab};
    for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; ++i) nnspk_free(bufs[i]);
    for (int i = 0; i < 3; ++i) nnspk_event_destroy(b->ev[i]);
    nnspk_stream_destroy(b->stream);
    free(b);
}

int nnsp_batch_reset(nnsp_batch *b, const uint8_t *mask)
{
    if (!b) return NNSP_EINVAL;
    const uint8_t *dm = NULL;
    if (mask) {
        TRY(nnspk_h2d(b->d_mask, mask, (size_t)b->S, b->stream));
        dm = b->d_mask;
    }
    /* FeatureClass_setDefault + NeuralNetClass_setDefault + NNSPClass fields */
    TRY(nnspk_launch_fe_default(b->d_prev5, b->d_tail, b->d_mean, b->d_stdR, b->norm_shift, dm, b->S,
                                b->stream));
    TRY(nnspk_launch_nn_default(b->d_h, b->d_c, b->d_post, (b->im.img.n_lstm ? b->im.img.n_lstm : 1) * b->hs,
                                dm, b->S, b->stream));
    return nnspk_sync(b->stream);
}

static int ensure(void **p, size_t bytes)
{
    if (*p) return 0;
    return nnspk_malloc(p, bytes);
}

int nnsp_batch_run(nnsp_batch *b, const int16_t *pcm, int T, int16_t *trig, int32_t *logits,
                   const nnsp_segment *seg, void *stream, int timed)
{
    static const nnsp_segment whole = {0};
    if (!seg) seg = &whole;
    if (seg->list && !b->fast) {
        nnsp_set_error("stream segments need the split NN path (one LSTM layer)");
        return NNSP_EUNSUPPORTED;
    }
    if (seg->list && seg->n_list <= 0) return 0;
    FeArgs fa;
    memset(&fa, 0, sizeof fa);
    fa.tb_img = b->d_fetab;
    fa.pcm = pcm;
    fa.tail = b->d_tail;
    fa.S = b->S;
    fa.T = T;
    fa.mean = b->d_mean;
    fa.stdR = b->d_stdR;
    fa.dbg_clk = b->d_clk;
    fa.norm_shift = b->norm_shift;
    fa.feats = b->d_feats;
    fa.list = seg->list;
    fa.n_list = seg->n_list;
    fa.seg_begin = seg->seg_begin;
    fa.lookback = seg->lookback;
    fa.hist = seg->hist;
    fa.hist_frames = seg->hist_frames;
    fa.seg_len = seg->seg_len;
    fa.port = b->port;
    fa.norm32 = b->norm32;
    if (timed) TRY(nnspk_event_record(b->ev[0], stream));
    TRY(nnspk_launch_fe(&fa, stream));
    if (timed) TRY(nnspk_event_record(b->ev[1], stream));
    TRY(nnsp_batch_run_nn(b, T, trig, logits, seg, stream));
    if (timed) TRY(nnspk_event_record(b->ev[2], stream));
    /* carry the PCM tail (last 320 samples) */
    TRY(nnspk_launch_tail_roll(b->d_tail, pcm, b->S, T, seg->list, seg->n_list, seg->seg_begin, seg->seg_len,
                               seg->lookback, seg->hist, seg->hist_frames, stream));
    return 0;
}

/* recur (compiled shapes): 16-stream tiles per workgroup, run back to back
 * through one pipeline -- its fill and drain (4 iterations) and the weight
 * staging once per workgroup instead of once per tile.  Short segments (a
 * cascade round's window) gain most; NNSP_RECUR_TSEQ=1..4 overrides. */
static int recur_tseq(const nnsp_segment *seg, int T, int shape)
{
    const char *e = getenv("NNSP_RECUR_TSEQ");   /* (read per launch: tests switch it) */
    int env = e ? atoi(e) : 0;
    if (shape == NN_SHAPE_VAD && (e = getenv("NNSP_RECUR_TSEQ_VAD")) != NULL) env = atoi(e);   /* development */
    if (env > 0) return env > 4 ? 4 : env;
    const int W = seg->seg_len > 0 && seg->seg_len < T ? seg->seg_len : T;
    const int steps = (W + 1) / 2;
    /* short segments: VAD 4 tiles per workgroup, S2I and KWS 2 (their
     * whole-CU pipelines: at 8 NN steps S2I's NN 1.35 -> 1.09 ms, KWS's 1.00 ->
     * 0.94 ms per chunk; synthetic-weight cascade 0.691 -> 0.701 G, paired,
     * profiles/r04/synth_tseq/) */
    if (steps <= 8 && shape == NN_SHAPE_VAD) return 4;
    return steps <= 16 ? 2 : 1;
}

int nnsp_batch_run_nn(nnsp_batch *b, int T, int16_t *trig, int32_t *logits, const nnsp_segment *seg,
                      void *stream)
{
    static const nnsp_segment whole = {0};
    if (!seg) seg = &whole;
    if (b->fast) {
        FastRun f;
        memset(&f, 0, sizeof f);
        f.S = b->S;
        f.T = T;
        f.li = b->li;
        f.nstep_max = b->nstep_max;
        f.feats = b->d_feats;
        f.prev5 = b->d_prev5;
        f.post = b->d_post;
        f.gx = b->d_gx;
        f.xg = b->d_xg;
        f.h = b->d_h;
        f.c = b->d_c;
        f.trig = trig;
        f.logits = logits;
        f.out3 = seg->out3;
        f.net_ran = seg->net_ran;
        f.detected = seg->detected;
        f.outputs3 = seg->outputs3;
        f.net_id = seg->net_id;
        f.fs = seg->fs;
        f.list = seg->list;
        f.n_list = seg->n_list;
        f.seg_begin = seg->seg_begin;
        f.seg_len = seg->seg_len;
        f.dbg_clk = seg->ctl && seg->ctl->round ? NULL : b->d_clk; /* probes: a cascade's round 0 */
        f.shape = b->shape;
        f.ep32 = b->ep32;
        const NnLayer *LL = &b->im.img.L[b->li];
        f.a_off = 0;
        f.a_lds_bytes = (int)(b->shape != NN_SHAPE_GENERIC ? LL->a_off : LL->ar_off);
        f.ep_lo = 0;
        f.ep_n = b->ep_proj;
        f.n_list_dev = seg->n_list_dev;
        f.n_list_rec = seg->n_list_rec;
        {   /* proj tiles: pack 2 or 4 streams per 16-row tile when a segment has <= 8 / 4 NN steps */
            const int W = seg->seg_len > 0 && seg->seg_len < T ? seg->seg_len : T;
            const int steps = (W + 1) / 2;
            /* (longer segments packed too -- 2 or 4 streams per tile, several
             * tiles per group, 12-19 % fewer tiles: cascade unchanged, VAD
             * NN 0.138 -> 0.143 ms; profiles/r03/gpt.sh) */
            f.gpt = b->shape == NN_SHAPE_GENERIC ? 1 : (steps <= 4 ? 4 : (steps <= 8 ? 2 : 1));
        }
        int blocks = b->proj_blocks;
        {   /* (NNSP_PROJ_LATE_BLOCKS, development: a smaller persistent grid for the
             * cascade's later rounds, whose device-sized lists are short) */
            static int late = -1;
            if (late < 0) {
                const char *e = getenv("NNSP_PROJ_LATE_BLOCKS");
                late = e && atoi(e) > 0 ? atoi(e) : 0;
            }
            if (late && seg->n_list_dev && seg->round > 0 && blocks > late) blocks = late;
        }
        if (seg->list && !seg->n_list_dev) {   /* size the grid to the listed streams */
            const int W = seg->seg_len > 0 && seg->seg_len < T ? seg->seg_len : T;
            const long long pt = (long long)seg->n_list * ((W / 2 + 1 + 15) / 16);
            const long long need = (pt + b->proj_waves - 1) / b->proj_waves;
            if (need < blocks) blocks = (int)need;
        }
        f.tseq = recur_tseq(seg, T, b->shape);
        /* the fused prefix: one tile per workgroup, features from the ring */
        const int fuse = b->fuse && f.tseq == 1 && seg->fs.nring != NULL;
        if (!fuse) TRY(nnspk_launch_proj(&b->im.img, &f, blocks, b->proj_waves, stream));
        if (seg->proj_done) TRY(nnspk_event_record(seg->proj_done, stream));
        for (int k = 0; k < 2; ++k)
            if (seg->recur_wait[k]) TRY(nnspk_stream_wait(stream, seg->recur_wait[k]));
        f.fuse = fuse;
        f.a_off = fuse ? 0 : b->rec_a_off;
        f.a_lds_bytes = (int)(b->im.a_bytes - (size_t)f.a_off);
        f.ep_lo = fuse ? 0 : b->ep_rec_lo;
        f.ep_n = fuse ? b->im.rows_total : b->ep_rec_n;
        TRY(nnspk_launch_recur(&b->im.img, &f, b->rec_waves, seg->ctl, stream));
    } else {
        NnRun r;
        memset(&r, 0, sizeof r);
        r.S = b->S;
        r.T = T;
        r.mode = NN_MODE_STREAM;
        r.nl_run = b->im.img.nl;
        r.feats = b->d_feats;
        r.prev5 = b->d_prev5;
        r.h = b->d_h;
        r.c = b->d_c;
        r.hs = b->hs;
        r.post = b->d_post;
        r.trig = trig;
        r.logits = logits;
        TRY(nnspk_launch_nn(&b->im.img, &r, stream));
        if (seg && seg->proj_done) TRY(nnspk_event_record(seg->proj_done, stream));
        /* carry the feature context (slots 1..5); recur_kernel does it on the split path */
        TRY(nnspk_launch_ctx_roll(b->d_prev5, b->d_feats, b->S, T, seg->list, seg->n_list, seg->seg_begin,
                                  seg->seg_len, stream));
    }
    return 0;
}

int nnsp_batch_exec_device(nnsp_batch *b, const int16_t *pcm, int T, int16_t *trig, int32_t *logits)
{
    if (!b || !pcm || T <= 0 || T > b->Tmax) {
        nnsp_set_error("nnsp_batch_exec: T must be in 1..%d", b ? b->Tmax : 0);
        return NNSP_EINVAL;
    }
    /* logits rows of frames without an NN step are defined as 0 */
    if (logits) TRY(nnspk_memset(logits, 0, (size_t)b->S * T * b->nout * 4, b->stream));
    TRY(nnsp_batch_run(b, pcm, T, trig, logits, NULL, b->stream, 1));
    b->last_T = T;
    return 0;
}

int nnsp_batch_exec(nnsp_batch *b, const int16_t *pcm, int T, int16_t *trig, int32_t *logits,
                    int16_t *features)
{
    if (!b || !pcm || T <= 0 || T > b->Tmax) return NNSP_EINVAL;
    const size_t S = (size_t)b->S;
    TRY(ensure((void **)&b->d_pcm, S * b->Tmax * 160 * 2));
    TRY(ensure((void **)&b->d_trig, S * b->Tmax * 2));
    if (logits) TRY(ensure((void **)&b->d_logits, S * b->Tmax * b->nout * 4));
    TRY(nnspk_h2d(b->d_pcm, pcm, S * T * 160 * 2, b->stream));
    TRY(nnsp_batch_exec_device(b, b->d_pcm, T, b->d_trig, logits ? b->d_logits : NULL));
    if (trig) TRY(nnspk_d2h(trig, b->d_trig, S * T * 2, b->stream));
    if (logits) TRY(nnspk_d2h(logits, b->d_logits, S * T * b->nout * 4, b->stream));
    if (features) TRY(nnspk_d2h(features, b->d_feats, S * T * 40 * 2, b->stream));
    return nnspk_sync(b->stream);
}

int nnsp_batch_sync(nnsp_batch *b) { return b ? nnspk_sync(b->stream) : NNSP_EINVAL; }
void *nnsp_batch_stream(nnsp_batch *b) { return b ? b->stream : NULL; }
int nnsp_batch_streams(const nnsp_batch *b) { return b ? b->S : 0; }
int nnsp_batch_nout(const nnsp_batch *b) { return b ? b->nout : 0; }
const int16_t *nnsp_batch_features_device(const nnsp_batch *b) { return b ? b->d_feats : NULL; }

int nnsp_batch_last_timing(nnsp_batch *b, float *fe_ms, float *nn_ms)
{
    if (!b) return NNSP_EINVAL;
    TRY(nnspk_sync(b->stream));
    TRY(nnspk_event_elapsed(fe_ms, b->ev[0], b->ev[1]));
    TRY(nnspk_event_elapsed(nn_ms, b->ev[1], b->ev[2]));
    return 0;
}

int nnsp_batch_post_state(nnsp_batch *b, nnsp_post_state *out)
{
    if (!b || !out) return NNSP_EINVAL;
    TRY(nnspk_d2h(out, b->d_post, (size_t)b->S * sizeof(NnPost), b->stream));
    return nnspk_sync(b->stream);
}

/* per-stream state blob: tail | prev5 | h | c | post */
size_t nnsp_batch_state_bytes(const nnsp_batch *b)
{
    const int nls = b->im.img.n_lstm ? b->im.img.n_lstm : 1;
    return 320 * 2 + 200 * 2 + (size_t)nls * b->hs * 6 + sizeof(NnPost);
}

static StateSeg plain_seg(const void *base, size_t stride, size_t bytes, size_t off)
{
    StateSeg g;
    memset(&g, 0, sizeof g);
    g.base = (unsigned long long)(uintptr_t)base;
    g.stride = stride;
    g.rows = 1;
    g.row_bytes = (uint32_t)bytes;
    g.wrap = 1;
    g.off = (uint32_t)off;
    return g;
}

int nnsp_batch_state_segs(const nnsp_batch *b, StateSeg *seg, size_t off, size_t *end)
{
    const int nls = b->im.img.n_lstm ? b->im.img.n_lstm : 1;
    const size_t hb = (size_t)nls * b->hs * 2, cb = (size_t)nls * b->hs * 4;
    seg[0] = plain_seg(b->d_tail, 640, 640, off);
    seg[1] = plain_seg(b->d_prev5, 400, 400, off + 640);
    seg[2] = plain_seg(b->d_h, hb, hb, off + 1040);
    seg[3] = plain_seg(b->d_c, cb, cb, off + 1040 + hb);
    seg[4] = plain_seg(b->d_post, sizeof(NnPost), sizeof(NnPost), off + 1040 + hb + cb);
    *end = off + nnsp_batch_state_bytes(b);
    return 5;
}

/* through one device staging buffer of at most NNSP_STATE_STAGE bytes, in
 * batches of streams: a whole large shard at once needed a transient
 * allocation of hundreds of MB, whose failure left the caller unable to
 * checkpoint */
#define NNSP_STATE_STAGE ((size_t)16 << 20)
int nnsp_state_xfer(StateCopy *sc, void *host, void *stream)
{
    if (sc->count == 0) return 0;
    const int first = sc->first, count = sc->count;
    size_t per_batch = NNSP_STATE_STAGE / sc->per;
    if (per_batch < 1) per_batch = 1;
    const int nb = (int)((size_t)count < per_batch ? (size_t)count : per_batch);
    void *d = NULL;
    int e = nnspk_malloc(&d, (size_t)nb * sc->per);
    if (e) return e;
    for (int i = 0; i < count && !e; i += nb) {
        const int k = count - i < nb ? count - i : nb;
        char *hb = (char *)host + (size_t)i * sc->per;
        const size_t n = (size_t)k * sc->per;
        sc->first = first + i;
        sc->count = k;
        if (!sc->to_blob) e = nnspk_h2d(d, hb, n, stream);
        if (!e) e = nnspk_launch_state_copy(sc, d, stream);
        if (!e && sc->to_blob) e = nnspk_d2h(hb, d, n, stream);
        if (!e) e = nnspk_sync(stream);
    }
    sc->first = first;
    sc->count = count;
    nnspk_free(d);
    return e;
}

static int state_xfer(nnsp_batch *b, void *host, int first, int count, int to_dev)
{
    if (!b || !host || first < 0 || count < 0 || first + count > b->S) return NNSP_EINVAL;
    StateCopy sc;
    memset(&sc, 0, sizeof sc);
    size_t end = 0;
    sc.nseg = nnsp_batch_state_segs(b, sc.seg, 0, &end);
    sc.per = end;
    sc.first = first;
    sc.count = count;
    sc.to_blob = !to_dev;
    return nnsp_state_xfer(&sc, host, b->stream);
}

int nnsp_batch_get_state(nnsp_batch *b, void *host, int first, int count)
{
    return state_xfer(b, host, first, count, 0);
}

int nnsp_batch_set_state(nnsp_batch *b, const void *host, int first, int count)
{
    return state_xfer(b, (void *)host, first, count, 1);
}

/* development probe (not in the public header): recur_kernel phase clocks of
 * tile 0 for the last chunk, [64 steps][8] s_memtime values */
int nnsp_batch_debug_clocks(nnsp_batch *b, long long *out)
{
    if (!b || !out || !b->d_clk) return NNSP_EINVAL;
    TRY(nnspk_d2h(out, b->d_clk, 64 * 32 * 8, b->stream));
    return nnspk_sync(b->stream);
}

/* development probe: zero the clock buffer (before an instrumented chunk) */
int nnsp_batch_debug_clocks_clear(nnsp_batch *b)
{
    if (!b || !b->d_clk) return NNSP_EINVAL;
    TRY(nnspk_memset(b->d_clk, 0, DCLK_LONGS * 8, b->stream));
    return nnspk_sync(b->stream);
}

/* development probe: the first n longs of the clock buffer (past the 2048 of
 * nnsp_batch_debug_clocks: fe_kernel's per-wave records, 4 longs per wave) */
int nnsp_batch_debug_clocks_n(nnsp_batch *b, long long *out, int n)
{
    if (!b || !out || !b->d_clk || n <= 0 || n > DCLK_LONGS) return NNSP_EINVAL;
    TRY(nnspk_d2h(out, b->d_clk, (size_t)n * 8, b->stream));
    return nnspk_sync(b->stream);
}

int nnsp_synth_pcm(int16_t *dev_out, int S, int T, uint64_t seed, int s0, int64_t t0, int amp, void *stream)
{
    if (!dev_out || S <= 0 || T <= 0 || amp <= 0) return NNSP_EINVAL;
    return nnspk_launch_synth_pcm(dev_out, S, T, (unsigned long long)seed, s0, (long long)t0, amp, NULL, 0, 0, 0,
                                  stream);
}

int nnsp_synth_pcm_mix(int16_t *dev_out, int S, int T, uint64_t seed, int s0, int64_t t0, int amp,
                       const int16_t *dev_wavs, int n_wavs, int wav_len, int every, void *stream)
{
    if (!dev_out || S <= 0 || T <= 0 || amp <= 0 || (dev_wavs && (n_wavs <= 0 || wav_len <= 0 || every <= 0)))
        return NNSP_EINVAL;
    return nnspk_launch_synth_pcm(dev_out, S, T, (unsigned long long)seed, s0, (long long)t0, amp, dev_wavs, n_wavs,
                                  wav_len, every, stream);
}
