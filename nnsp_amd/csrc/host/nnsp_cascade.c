/*
 * nnsp_cascade.c -- batched nnCntrlClass (include/nnsp_cascade.h).
 *
 * Per chunk:
 *   1. one front-end launch computes the log-Mel of every PCM frame of every
 *      stream (FE_MODE_SHARED) into a ring that also keeps the look-back
 *      frames of earlier chunks.  The log-Mel of a frame does not depend on
 *      the net: all three nets run the same FeatureClass up to log10_vec, and
 *      a net whose STFT buffer holds the real previous frames sees exactly the
 *      shared value of the frame it reads (the current one for VAD, the one
 *      frs_vbufBk frames back for KWS / S2I);
 *   2. casc_begin lists every stream under the net at its position;
 *   3. rounds of { for each net with listed streams, on its own HIP stream:
 *      the full front end of the 0-2 frames right after the net's reset,
 *      whose STFT buffer still holds zeros (FE_MODE_COLD; every other frame's
 *      features are the shared log-Mel normalised on the fly by the kernels
 *      that read them), then the NN half (proj -> recur).  recur runs the
 *      controller as the triggers come out, cuts each stream's segment at its
 *      first net switch, stores the departing net's reset state and lists the
 *      stream for the next round } until no stream is listed;
 *   4. the shared front end's PCM tail rolls forward (the PCM history that
 *      the look-back and the cold frames read was stored by step 1).
 * The host reads back three list lengths per batch of rounds and nothing else.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../../include/nnsp_cascade.h"
#include "nnsp_host.h"

/* NNSP_CASCADE_DEBUG: after each launch, wait for the stream and report
 * which launch failed (asynchronous faults otherwise surface at a later sync) */
static int dbg_step(const nnsp_cascade *c, void *stream, const char *what, int n, int r);
static void zero_bind(nnsp_cascade *c, int parity);
static int book_take(nnsp_cascade *c);
static int ahead_read(nnsp_cascade *c, int q, int wait);
#define DBG(st, what, n, r)                                  \
    do {                                                     \
        if (c->debug) TRY(dbg_step(c, (st), (what), (n), (r))); \
    } while (0)

#define TRY(x)                 \
    do {                       \
        int _e = (x);          \
        if (_e) return _e;     \
    } while (0)

#define HIST_MAX 99   /* PcmBufClass keeps 100 frames: look-back 0..99 */
#define MAX_TIMED 32  /* rounds per chunk with per-net device timing */
#define ZERO_BYTES (3 * 8 + (18 + 2 + MAX_TIMED * 3) * 4)
#define ZERO_STRIDE 512   /* the counters of chunk parity p at d_zero + p * ZERO_STRIDE */
_Static_assert(ZERO_BYTES <= ZERO_STRIDE, "the two chunk-parity counter blocks overlap: raise ZERO_STRIDE");

struct nnsp_cascade {
    nnsp_batch *net[3];
    int S, Tmax, H;
    int lookback[3];
    CascArgs a;                     /* persistent device pointers */
    CascState *d_st;
    int32_t *d_seg_begin, *d_counts;
    unsigned long long *d_frames;
    int16_t *d_trig[3];             /* per net: triggers for casc_control (control-kernel mode only) */
    uint8_t *d_mask[3];
    /* per round parity and net: the round's stream lists (round r reads
     * [r & 1] while its kernels append the next round's to [(r + 1) & 1]) */
    int32_t *d_list[2][3], *d_cold_list[2][3];
    int16_t *d_hist[3];             /* PCM history before chunk k: d_hist[k % 3] (the look-ahead
                                       front end of chunk k+1 writes d_hist[(k + 2) % 3]) */
    long long chunk;                /* chunks run since create */
    int debug;                      /* NNSP_CASCADE_DEBUG: synchronise after every launch, name the failing one */
    int16_t *d_nring[3];            /* per net id: [S][ring][40] normalised shared front-end output */
    int ring, abs0;                 /* ring slots (>= H + Tmax); slot of chunk frame 0 */
    int16_t *d_stail;               /* [S][320] PCM tail of the shared front end */
    int8_t *d_fresh;                /* [S] frames the current net ran since its reset */
    int16_t *d_pcm, *d_det, *d_o3;
    int8_t *d_ran;
    int16_t *d_pdef;                /* [3][40] FeatureClass_setDefault context value per net */
    int32_t *d_rcount;              /* [MAX_TIMED][3] list lengths each round ran with */
    int32_t *d_last_round;          /* last round a stream was listed for (+1) */
    int32_t *d_cuts;                /* segments cut by a net switch in the chunk */
    void *d_fetab;                  /* the shared / cold front end's tables, prebuilt */
    int fe_sched;                   /* the shared front end's frame schedule (FE_SCHED_*) */
    void *d_zero;                   /* frames, counts, last_round, rcount (one allocation), per chunk parity:
                                       chunk k counts into block k & 1 and clears block (k + 1) & 1 */
    void *stream;                   /* front end, control; the nets' work forks off it */
    void *bstream;                  /* early return: the chunk's join and counter copy, beside the look-ahead
                                       front end on c->stream */
    int early;                      /* return once the rounds are done, before the look-ahead front end ends
                                       (the next call's round 0 waits for it on the device) */
    int early_prev;                 /* the last call returned early */
    void *ns[3];                    /* per net id: segment features + NN of a round */
    void *own_ns[3];                /* per net id: a cascade-owned high-priority stream used as ns[n]
                                       (NNSP_NET_PRIO bit n, development), else NULL */
    void *ev[2];
    void *ev_fe[2];                 /* shared front end */
    void *ev_fork, *ev_join[3];
    void *ev_vad_proj;              /* VAD's round-0 prefix FC layers done */
    void *ev_r0proj[3];             /* round-0 prefix FC layers done, per net (r0_order 3) */
    void *ev_r1proj[3];             /* round-1 prefix FC layers done, per net (ahead_mode 1) */
    int ahead_mode;                 /* when the look-ahead front end starts (NNSP_AHEAD_MODE, see exec) */
    int r0_order;                   /* round 0's launch order (NNSP_R0_ORDER, see launch_round) */
    int8_t seq[8];                  /* pt_seq_cntrl: NNSP_ID per sequence position */
    int len_seq;
    void *ev_rnd[2][3];             /* fused control: per round parity and net, end of the net's round */
    void *ev_t[MAX_TIMED][3][3];    /* per round and net: before features, before NN, after NN */
    int last_rounds, launched;
    /* running totals since create / nnsp_cascade_totals_reset (nnsp_cascade_totals) */
    long long tot_chunks, tot_rounds;
    unsigned long long tot_frames;
    double tot_fe_ms, tot_chunk_ms;
    const int16_t *pre_pcm;         /* the chunk whose shared front end the last call ran ahead */
    int pre_T;
    /* look-ahead front end of chunk q (events by chunk parity q & 1: around
     * the launch; read without waiting once it has finished, or by sync) */
    void *ev_ahead[2][2];
    int ahead_pending[2];
    float ahead_ms[2];
    int sfe_ahead;                  /* last chunk's shared front end ran in the previous call */
    int window;                     /* frames per stream and round (0: to the chunk end) */
    int auto_window;                /* pick window per chunk from the last chunk's switch rate */
    int last_cuts;                  /* last chunk: segments cut by a net switch */
    int serial;                     /* NNSP_CASCADE_SERIAL: the nets' work on the main stream (no fork/join) */
    int fused;                      /* controller fused into the nets' recur kernels (compiled shapes) */
    int timing;                     /* per-round, per-net device timing (set_timing; NNSP_CASCADE_TIMING) */
    float sfe_ms;                   /* last chunk: shared front end */
    float fe_ms[3], nn_ms[3];       /* last chunk, per net id: features / proj+recur+roll */
    int runs[3];                    /* last chunk, per net id: segment runs */
    int rc[MAX_TIMED][3];           /* last chunk: list length of each round and net */
    float rfe[MAX_TIMED][3], rnn[MAX_TIMED][3]; /* last chunk, timing on: per round and net ms */
    /* end-of-chunk bookkeeping, asynchronous: the chunk's counters (d_zero) are
     * copied to pinned host memory and cleared for the next chunk on the
     * stream; the host reads the copy (book_take) when it next needs it */
    void *h_book;                   /* pinned copy of d_zero */
    void *ev_book;                  /* recorded after the copy */
    int book_pending;               /* a copy is in flight */
    int book_rounds;                /* rounds launched in that chunk */
    int book_ahead, book_ahead_done; /* its look-ahead front end ran; its own front end ran ahead */
    int chunk_open;                 /* a call launched rounds and did not finish: its parity block holds
                                       partial counts (cleared by the next call before use) */
    unsigned long long book_frames[3];
};

/* the chunk counters of parity p (c->d_* and the kernels' CascArgs pointers) */
static void zero_bind(nnsp_cascade *c, int parity)
{
    char *z = (char *)c->d_zero + (size_t)parity * ZERO_STRIDE;
    c->d_frames = (unsigned long long *)z;              /* [3] */
    c->d_counts = (int32_t *)(z + 3 * 8);               /* [18] */
    c->d_last_round = c->d_counts + 18;                 /* [1] */
    c->d_cuts = c->d_last_round + 1;                    /* [1] */
    c->d_rcount = c->d_cuts + 1;                        /* [MAX_TIMED][3] */
    c->a.counts = c->d_counts;
    c->a.frames = c->d_frames;
    c->a.last_round = c->d_last_round;
    c->a.cuts = c->d_cuts;
}

int nnsp_cascade_create(nnsp_cascade **out, nnsp_batch *const nets[3], const int8_t *seq, int len_seq,
                        const nnsp_cascade_params *p)
{
    *out = NULL;
    if (!nets || !seq || !p || len_seq < 1 || len_seq > 8) {
        nnsp_set_error("nnsp_cascade_create: bad argument");
        return NNSP_EINVAL;
    }
    for (int i = 0; i < 3; ++i) {
        if (!nets[i] || nets[i]->S != nets[0]->S) {
            nnsp_set_error("nnsp_cascade_create: three nets of the same stream count required");
            return NNSP_EINVAL;
        }
        if (nets[i]->port != nets[0]->port) {
            nnsp_set_error("nnsp_cascade_create: nets of different builds (ARM_OPTIMIZED 1 and 0) share one front end");
            return NNSP_EINVAL;
        }
        if (nets[i]->nn_id != i) {
            nnsp_set_error("nnsp_cascade_create: nets[%d] was created with NNSP_ID %d (nets[] is indexed by NNSP_ID: "
                           "0 s2i, 1 vad, 2 kws)", i, nets[i]->nn_id);
            return NNSP_EINVAL;
        }
        if (!nets[i]->fast) {
            nnsp_set_error("nnsp_cascade_create: net %d has no split NN path (one LSTM layer)", i);
            return NNSP_EUNSUPPORTED;
        }
    }
    for (int i = 0; i < len_seq; ++i)
        if (seq[i] < 0 || seq[i] > 2) {
            nnsp_set_error("nnsp_cascade_create: seq[%d] = %d is not an NNSP_ID", i, seq[i]);
            return NNSP_EINVAL;
        }
    if (p->frs_vbufBk_s2i < 0 || p->frs_vbufBk_s2i > HIST_MAX || p->frs_vbufBk_kws < 0 ||
        p->frs_vbufBk_kws > HIST_MAX || p->thresh_timeout_s2i < 1 || p->thresh_timeout_kws < 1) {
        nnsp_set_error("nnsp_cascade_create: look-back must be 0..%d, timeouts >= 1", HIST_MAX);
        return NNSP_EINVAL;
    }
    nnsp_cascade *c = (nnsp_cascade *)calloc(1, sizeof *c);
    if (!c) return NNSP_ENOMEM;
    *out = c;
    int e = 0;
    c->S = nets[0]->S;
    c->Tmax = nets[0]->Tmax;
    for (int i = 0; i < 3; ++i) {
        c->net[i] = nets[i];
        if (nets[i]->Tmax < c->Tmax) c->Tmax = nets[i]->Tmax;
    }
    memcpy(c->seq, seq, (size_t)len_seq);
    c->len_seq = len_seq;
    c->lookback[0] = p->frs_vbufBk_s2i;
    c->lookback[1] = 0; /* VAD reads the current frame (nnCntrlClass.c:243-247) */
    c->lookback[2] = p->frs_vbufBk_kws;
    /* PCM history: the look-back frame and, for the second frame after a
     * net's reset, the one before it (FE_MODE_COLD re-reads it); and one
     * more, the oldest frame in the STFT buffer of a net that runs at the
     * largest look-back (stftModule.dataBuffer[160..319]): the stream state
     * then maps onto the reference's own structs and back exactly
     * (nnsp_cascade_get_state_ref / set_state_ref) */
    c->H = (c->lookback[0] > c->lookback[2] ? c->lookback[0] : c->lookback[2]) + 2;
    c->ring = c->H + 2 * c->Tmax;   /* look-back + this chunk + the look-ahead chunk */
    /* ring rows s * ring + slot are 32-bit in the kernels (fe_kernel's shared
     * store, the proj union loads); element offsets beyond are 64-bit */
    if ((long long)c->S * c->ring >= (1LL << 31)) {
        nnsp_set_error("nnsp_cascade_create: streams * (look-back + 2 * max_frames) = %lld ring rows, must stay "
                       "below 2^31", (long long)c->S * c->ring);
        free(c);
        *out = NULL;
        return NNSP_EINVAL;
    }
    const size_t S = (size_t)c->S, T = (size_t)c->Tmax;
    if ((e = nnspk_stream_create(&c->stream))) goto fail;
    for (int i = 0; i < 2; ++i)
        if ((e = nnspk_event_create(&c->ev[i])) || (e = nnspk_event_create(&c->ev_fe[i]))) goto fail;
    /* the events that only order streams (and the host's wait on the counter
     * copy) carry no timestamps: the waits behind them resolve sooner (gaps
     * between rounds 20-24 -> 13-20 us in the stress case's kernel trace;
     * cascade 1.2454 -> 1.2569 and 1.2196 -> 1.2358 G, 9 of 11 pairs,
     * profiles/r05/dep_events/).  NNSP_DEP_EVENTS=0: timed events throughout */
    const char *dv = getenv("NNSP_DEP_EVENTS");
    const int dep = dv ? atoi(dv) : 1;
#define DEP_EVENT(p) (dep ? nnspk_event_create_dep(p) : nnspk_event_create(p))
    if ((e = DEP_EVENT(&c->ev_fork))) goto fail;
    for (int q = 0; q < 2; ++q)
        if ((e = nnspk_event_create(&c->ev_ahead[q][0])) || (e = nnspk_event_create(&c->ev_ahead[q][1]))) goto fail;
    if ((e = DEP_EVENT(&c->ev_vad_proj))) goto fail;
    for (int n = 0; n < 3; ++n)
        if ((e = DEP_EVENT(&c->ev_r0proj[n])) || (e = DEP_EVENT(&c->ev_r1proj[n]))) goto fail;
    for (int n = 0; n < 3; ++n) {
        /* each net's rounds run on its batch's own stream: the cascade adds
         * one stream (c->stream) to the three, so on a device with four
         * hardware queues (HIP's default) the look-ahead front end on
         * c->stream never shares an in-order queue with a net's rounds */
        c->ns[n] = nets[n]->stream;
        {   /* NNSP_NET_PRIO (development): bit n = net n's rounds on a high-priority stream of the
             * cascade's own, so that its workgroups are dispatched ahead of the other nets' */
            const char *pe = getenv("NNSP_NET_PRIO");
            if (pe && (atoi(pe) >> n) & 1) {
                if ((e = nnspk_stream_create_prio(&c->own_ns[n], 1))) goto fail;
                c->ns[n] = c->own_ns[n];
            }
        }
        if ((e = DEP_EVENT(&c->ev_join[n])) || (e = DEP_EVENT(&c->ev_rnd[0][n])) || (e = DEP_EVENT(&c->ev_rnd[1][n])))
            goto fail;
        for (int r = 0; r < MAX_TIMED; ++r)
            for (int i = 0; i < 3; ++i)
                if ((e = nnspk_event_create(&c->ev_t[r][n][i]))) goto fail;
    }
    if ((e = nnspk_malloc((void **)&c->d_st, S * sizeof(CascState)))) goto fail;
    /* the per-chunk counters, one allocation zeroed by one memset per chunk */
    if ((e = nnspk_malloc((void **)&c->d_zero, 2 * ZERO_STRIDE))) goto fail;
    if ((e = nnspk_memset(c->d_zero, 0, 2 * ZERO_STRIDE, c->stream))) goto fail;
    if ((e = nnspk_host_alloc(&c->h_book, ZERO_BYTES))) goto fail;
    if ((e = DEP_EVENT(&c->ev_book))) goto fail;
#undef DEP_EVENT
    zero_bind(c, 0);
    if ((e = nnspk_malloc((void **)&c->d_seg_begin, S * 4))) goto fail;
    /* list lengths of 3 rounds in flight: 3 lists + 3 cold lists each */
    if ((e = nnspk_malloc((void **)&c->d_pdef, 3 * 40 * 2))) goto fail;
    /* the three rings in one allocation, ring n at n * S * ring * 40: the
     * shared front end then stores through one base pointer */
    if ((e = nnspk_malloc((void **)&c->d_nring[0], 3 * S * (size_t)c->ring * 40 * 2))) goto fail;
    for (int i = 1; i < 3; ++i) c->d_nring[i] = c->d_nring[0] + (size_t)i * S * c->ring * 40;
    if ((e = nnspk_malloc((void **)&c->d_stail, S * 640))) goto fail;
    {   /* the shared front end's frame schedule (FE_SCHED_*; NNSP_FE_SCHED, development) */
        const char *fs = getenv("NNSP_FE_SCHED");
        c->fe_sched = fs ? atoi(fs) : FE_SCHED_GUIDED;
        const char *fg = getenv("NNSP_FE_GUIDE"); /* "twelfths,divisor" of the guided schedule */
        if (fg && c->fe_sched == FE_SCHED_GUIDED) {
            int g12 = 0, dv = 0;
            if (sscanf(fg, "%d,%d", &g12, &dv) == 2 && g12 > 0 && g12 < 12 && dv > 0 && dv < 256)
                c->fe_sched |= (g12 << 8) | (dv << 16);
        }
    }
    /* (rounded up to whole dwords: proj DMAs the dword holding a stream's byte) */
    if ((e = nnspk_malloc((void **)&c->d_fresh, ((size_t)S + 3) & ~(size_t)3))) goto fail;
    for (int i = 0; i < 3; ++i) {
        if ((e = nnspk_malloc((void **)&c->d_trig[i], S * T * 2))) goto fail;
        if ((e = nnspk_malloc((void **)&c->d_mask[i], S))) goto fail;
        for (int k = 0; k < 2; ++k) {
            if ((e = nnspk_malloc((void **)&c->d_list[k][i], S * 4))) goto fail;
            if ((e = nnspk_malloc((void **)&c->d_cold_list[k][i], S * 4))) goto fail;
        }
        if ((e = nnspk_memset(c->d_mask[i], 0, S, c->stream))) goto fail;
    }
    for (int i = 0; i < 3; ++i)
        if ((e = nnspk_malloc((void **)&c->d_hist[i], S * (size_t)c->H * 320))) goto fail;
    if ((e = nnspk_memset(c->d_st, 0, S * sizeof(CascState), c->stream))) goto fail; /* pos 0 */
    {
        CascArgs *a = &c->a;
        memset(a, 0, sizeof *a);
        a->S = c->S;
        a->len_seq = len_seq;
        a->timeout_kws = p->thresh_timeout_kws;
        a->timeout_s2i = p->thresh_timeout_s2i;
        for (int i = 0; i < len_seq; ++i) {
            a->seq[i] = seq[i];
            a->seq_bits |= (int32_t)seq[i] << (2 * i);
        }
        a->st = c->d_st;
        a->seg_begin = c->d_seg_begin;
        a->counts = c->d_counts;
        a->frames = c->d_frames;
        a->fresh = c->d_fresh;
        a->last_round = c->d_last_round;
        a->cuts = c->d_cuts;
        for (int i = 0; i < 3; ++i) {
            a->trig[i] = c->d_trig[i];
            a->feats[i] = nets[i]->d_feats;
            a->prev5[i] = nets[i]->d_prev5;
            a->h[i] = nets[i]->d_h;
            a->c[i] = nets[i]->d_c;
            a->post[i] = nets[i]->d_post;
            a->prev_default[i] = c->d_pdef + 40 * i;
            a->list[i] = c->d_list[0][i]; /* round 0 (casc_begin); set per round */
            a->cold_list[i] = c->d_cold_list[0][i];
            FeatSrc *fs = &a->fs[i];
            fs->nring = c->d_nring[i];
            fs->fresh = c->d_fresh;
            fs->ring = c->ring;
            fs->lookback = c->lookback[i];
        }
    }
    {   /* the reset context value of each net: FeatureClass_setDefault on a scratch stream */
        int16_t *p5 = NULL, *tl = NULL;
        if ((e = nnspk_malloc((void **)&p5, 400)) || (e = nnspk_malloc((void **)&tl, 640))) {
            nnspk_free(p5);
            goto fail;
        }
        for (int i = 0; i < 3 && !e; ++i) {
            nnsp_batch *b = nets[i];
            e = nnspk_launch_fe_default(p5, tl, b->d_mean, b->d_stdR, b->norm_shift, NULL, 1, c->stream);
            if (!e) e = nnspk_d2d(c->d_pdef + 40 * i, p5, 80, c->stream);
        }
        if (!e) e = nnspk_sync(c->stream);
        nnspk_free(p5);
        nnspk_free(tl);
        if (e) goto fail;
    }
    {   /* the front end's tables: the shared mode's, with each net's normalisation (the cold mode reads none of those) */
        FeArgs ta;
        memset(&ta, 0, sizeof ta);
        ta.mode = FE_MODE_SHARED;
        ta.port = nets[0]->port;
        for (int n = 0; n < 3; ++n) {
            ta.nring[n] = c->d_nring[n];
            ta.nmean[n] = nets[n]->d_mean;
            ta.nstdR[n] = nets[n]->d_stdR;
        }
        if ((e = nnspk_build_fe_tables(&c->d_fetab, &ta, c->stream))) goto fail;
    }
    c->window = 16;      /* the first chunk's window; then chosen per chunk (auto_window) */
    c->auto_window = 1;
    {
        c->serial = getenv("NNSP_CASCADE_SERIAL") != NULL;
        {
            const char *o = getenv("NNSP_R0_ORDER");
            c->r0_order = o ? atoi(o) : 6;
            const char *am = getenv("NNSP_AHEAD_MODE");
            c->ahead_mode = am ? atoi(am) : 1;
        }
        /* the controller runs inside the nets' pipelined recur kernels when all
         * three have compiled shapes (NNSP_CASCADE_CONTROL_KERNEL: a separate
         * casc_control launch per round instead).  Serial mode keeps it: the
         * cross-net event waits are then waits on the same stream. */
        c->fused = getenv("NNSP_CASCADE_CONTROL_KERNEL") == NULL;
        for (int i = 0; i < 3; ++i)
            if (nets[i]->shape == NN_SHAPE_GENERIC) c->fused = 0;
        c->timing = getenv("NNSP_CASCADE_TIMING") != NULL;
        {
            const char *er = getenv("NNSP_EARLY_RETURN");
            c->early = er ? atoi(er) != 0 : 0;
            /* its book stream only when used: HIP has four hardware queues per
             * process (GPU_MAX_HW_QUEUES), and the cascade and its nets hold four */
            if (c->early && (e = nnspk_stream_create(&c->bstream))) goto fail;
        }
        c->debug = getenv("NNSP_CASCADE_DEBUG") != NULL;
        const char *w = getenv("NNSP_CASCADE_WINDOW");
        if (w && atoi(w) >= 0) {
            c->window = atoi(w);
            c->auto_window = 0;
        }
    }
    if ((e = nnsp_cascade_reset(c, NULL))) goto fail;
    return 0;
fail:
    nnsp_cascade_destroy(c);
    *out = NULL;
    return e;
}

void nnsp_cascade_destroy(nnsp_cascade *c)
{
    if (!c) return;
    if (c->stream) nnspk_sync(c->stream);
    void *bufs[] = {c->d_st,      c->d_seg_begin, c->d_zero,    c->d_trig[0], c->d_trig[1],
                    c->d_trig[2], c->d_mask[0],   c->d_mask[1],
                    c->d_mask[2], c->d_list[0][0], c->d_list[0][1], c->d_list[0][2], c->d_hist[0], c->d_hist[1], c->d_hist[2],
                    c->d_nring[0], c->d_stail,     c->d_fresh,   c->d_pcm,     c->d_det,     c->d_o3,
                    c->d_ran,     c->d_pdef,      c->d_cold_list[0][0],
                    c->d_cold_list[0][1], c->d_cold_list[0][2], c->d_list[1][0], c->d_list[1][1], c->d_list[1][2],
                    c->d_cold_list[1][0], c->d_cold_list[1][1], c->d_cold_list[1][2], c->d_fetab};
    for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; ++i) nnspk_free(bufs[i]);
    for (int i = 0; i < 2; ++i) {
        nnspk_event_destroy(c->ev[i]);
        nnspk_event_destroy(c->ev_fe[i]);
    }
    nnspk_event_destroy(c->ev_fork);
    nnspk_event_destroy(c->ev_vad_proj);
    for (int n = 0; n < 3; ++n) {
        nnspk_event_destroy(c->ev_r0proj[n]);
        nnspk_event_destroy(c->ev_r1proj[n]);
    }
    for (int q = 0; q < 2; ++q) {
        nnspk_event_destroy(c->ev_ahead[q][0]);
        nnspk_event_destroy(c->ev_ahead[q][1]);
    }
    for (int n = 0; n < 3; ++n) {
        nnspk_event_destroy(c->ev_join[n]);
        nnspk_event_destroy(c->ev_rnd[0][n]);
        nnspk_event_destroy(c->ev_rnd[1][n]);
        for (int r = 0; r < MAX_TIMED; ++r)
            for (int i = 0; i < 3; ++i) nnspk_event_destroy(c->ev_t[r][n][i]);
        c->ns[n] = NULL; /* the batch's stream, owned by the batch (or own_ns[n]) */
        if (c->own_ns[n]) {
            nnspk_sync(c->own_ns[n]);
            nnspk_stream_destroy(c->own_ns[n]);
        }
    }
    if (c->bstream) nnspk_sync(c->bstream);
    nnspk_stream_destroy(c->stream);
    nnspk_stream_destroy(c->bstream);
    nnspk_event_destroy(c->ev_book);
    nnspk_host_free(c->h_book);
    free(c);
}

int nnsp_cascade_reset(nnsp_cascade *c, const uint8_t *mask)
{
    if (!c) return NNSP_EINVAL;
    TRY(nnspk_sync(c->stream));
    TRY(book_take(c));
    for (int i = 0; i < 3; ++i) TRY(nnsp_batch_reset(c->net[i], mask)); /* synchronous */
    const uint8_t *dm = NULL;
    if (mask) {
        TRY(nnspk_h2d(c->d_mask[0], mask, (size_t)c->S, c->stream));
        dm = c->d_mask[0];
    }
    c->pre_pcm = NULL; /* a look-ahead front end ran on the old tail: recompute */
    /* both chunk-parity counter blocks: a failed call may have left partial counts */
    TRY(nnspk_memset(c->d_zero, 0, 2 * ZERO_STRIDE, c->stream));
    c->chunk_open = 0;
    TRY(nnspk_launch_casc_reset(c->d_st, c->d_hist[c->chunk % 3], c->H, c->d_stail, c->d_fresh, dm, c->S,
                                c->stream));
    /* PcmBufClass_reset: every look-back frame is silence */
    {
        const int32_t *mn[3], *sd[3];
        int32_t sh[3];
        for (int n = 0; n < 3; ++n) {
            mn[n] = c->net[n]->d_mean;
            sd[n] = c->net[n]->d_stdR;
            sh[n] = c->net[n]->norm_shift;
        }
        TRY(nnspk_launch_nring_fill(c->d_nring, mn, sd, sh, c->ring, dm, c->S, c->stream));
    }
    if (mask) TRY(nnspk_memset(c->d_mask[0], 0, (size_t)c->S, c->stream));
    return nnspk_sync(c->stream);
}

/* features of net n for this round's segments: the full front end for the
 * frames right after the net's reset (the others are normalised from the
 * shared log-Mel by the kernels that read them, FeatSrc) */
static int dbg_step(const nnsp_cascade *c, void *stream, const char *what, int n, int r)
{
    (void)c;
    const int e = nnspk_sync(stream);
    if (e) {
        fprintf(stderr, "nnsp_cascade: %s (net %d, round %d) failed: %s\n", what, n, r, nnspk_error_string(e));
        nnsp_set_error("nnsp_cascade: %s (net %d, round %d) failed", what, n, r);
    }
    return e;
}

static int segment_features(nnsp_cascade *c, int n, int r, const int16_t *pcm, int T, const int32_t *cnt,
                            const int16_t *hist, void *stream)
{
    nnsp_batch *b = c->net[n];
    FeArgs fa;
    memset(&fa, 0, sizeof fa);
    fa.tb_img = c->d_fetab;
    fa.pcm = pcm;
    fa.S = c->S;
    fa.T = T;
    fa.mean = b->d_mean;
    fa.stdR = b->d_stdR;
    fa.norm_shift = b->norm_shift;
    fa.feats = b->d_feats;
    fa.list = c->d_list[r & 1][n];
    fa.n_list_dev = cnt + n;
    fa.seg_begin = c->d_seg_begin;
    fa.lookback = c->lookback[n];
    fa.hist = hist;
    fa.hist_frames = c->H;
    fa.seg_len = c->window;
    fa.ring = c->ring;
    fa.abs0 = c->abs0;
    fa.fresh = c->d_fresh;
    fa.mode = FE_MODE_COLD;
    fa.port = b->port;
    fa.norm32 = b->norm32;
    fa.list = c->d_cold_list[r & 1][n];
    fa.n_list_dev = cnt + 3 + n;
    return nnspk_launch_fe(&fa, stream);
}

/* net n's NN kernels of round r on stream st (after its cold front end);
 * wait_cold: first wait for the other nets' cold front ends (ev_join) */
static int round_nn(nnsp_cascade *c, CascArgs *a, int r, int n, int T, int32_t *cur, const int16_t *hist, void *st,
                    void *proj_done, void *recur_wait0, void *recur_wait1)
{
    const int timed = c->timing && r < MAX_TIMED;
    nnsp_segment seg;
    memset(&seg, 0, sizeof seg);
    seg.proj_done = proj_done;
    seg.recur_wait[0] = recur_wait0;
    seg.recur_wait[1] = recur_wait1;
    seg.round = r;
    seg.list = c->d_list[r & 1][n];
    seg.n_list_dev = cur + n;
    seg.seg_begin = c->d_seg_begin;
    seg.lookback = c->lookback[n];
    seg.hist = hist;
    seg.hist_frames = c->H;
    seg.seg_len = c->window;
    seg.net_ran = a->net_ran;
    seg.detected = a->detected;
    seg.outputs3 = a->outputs3;
    seg.net_id = n;
    seg.fs = a->fs[n];
    seg.n_list_rec = r < MAX_TIMED ? c->d_rcount + 3 * r + n : NULL;
    seg.ctl = c->fused ? a : NULL;
    TRY(nnsp_batch_run_nn(c->net[n], T, c->fused ? NULL : c->d_trig[n], NULL, &seg, st));
    DBG(st, "proj + recur", n, r);
    if (timed) TRY(nnspk_event_record(c->ev_t[r][n][2], st));
    if (c->fused) {
        TRY(nnspk_event_record(c->ev_rnd[r & 1][n], st));
    } else if (!c->serial) {
        TRY(nnspk_event_record(c->ev_join[n], st));
        TRY(nnspk_stream_wait(c->stream, c->ev_join[n]));
    }
    return 0;
}

/* One round, asynchronous: the three nets' segments on their own streams
 * (empty lists exit on the device).  Fused control: each net's recur kernel
 * runs the controller for its streams and lists them for the next round, so
 * a net's next round waits only for the other two nets' end of this round.
 * Otherwise: join, casc_control on the main stream, fork. */
static int launch_round(nnsp_cascade *c, CascArgs *a, int r, const int16_t *pcm, int T, const int16_t *hist)
{
    int32_t *cur = c->d_counts + 6 * (r % 3);
    a->counts = c->d_counts + 6 * ((r + 1) % 3);
    a->counts_clear = c->d_counts + 6 * ((r + 2) % 3);
    a->round = r;
    for (int n = 0; n < 3; ++n) {
        a->list[n] = c->d_list[(r + 1) & 1][n];
        a->cold_list[n] = c->d_cold_list[(r + 1) & 1][n];
    }
    if (!c->serial && !c->fused) TRY(nnspk_event_record(c->ev_fork, c->stream));
    /* (measured and dropped, profiles/r02/sched: every net's cold front end
     * of a round before any net's NN kernels, VAD's recurrence after S2I's
     * and KWS's, every recur behind all three projs -- each -2..-7 %) */
    /* round 0 with fused control: until round 5, VAD (net 1) was launched first.  Until round
     * 4 S2I's and KWS's proj + recur waited for VAD's proj (r0_order 0;
     * profiles/r03: +1 % then).  With the faster proj and recurrences of
     * round 4 that wait only delayed S2I's and KWS's proj until VAD's 2 048
     * recurrence workgroups held every CU (KWS proj 164 -> 524 us, the round's
     * critical path); without it (r0_order 1) round 0 ends ~70 us earlier:
     * 1.080 vs 1.062 G (3 runs each), profiles/r04/r0_order/. */
    /* round 5: S2I first (r0_order 6, the default since; its recurrence is the
     * round's critical chain, trace in profiles/r05/chunk_trace): 1.2602 vs
     * 1.2554 G, every one of 6 pairs, and 4 of 4 in another pass
     * (profiles/r05/r0_order/).  casc_begin stays on VAD's stream: on S2I's or
     * KWS's it measured 1.09 vs 1.21 G (profiles/r05/r0_order/begin_net/) */
    /* r0_order (NNSP_R0_ORDER, development): 0 S2I's and KWS's NN wait for
     * VAD's proj; 1 VAD launched first, nothing waits; 3 S2I and
     * KWS launched first, VAD's recurrence waits for their proj (1.059 G);
     * 4 KWS, S2I, VAD, 5 VAD, KWS, S2I, 6 S2I, VAD, KWS and 7 S2I, KWS, VAD,
     * nothing waits */
    static const int o_plain[3] = {0, 1, 2}, o_vad[3] = {1, 0, 2}, o_vad_last[3] = {0, 2, 1};
    static const int o_kws_first[3] = {2, 0, 1}, o_vad_kws[3] = {1, 2, 0};
    const int r0 = r == 0 && c->fused && !c->serial;
    const int vad_first = r0 && c->r0_order == 0;
    const int vad_last = r0 && c->r0_order == 3;
    const int *order = vad_last || (r0 && c->r0_order == 7) ? o_vad_last
                     : (r0 && c->r0_order == 4 ? o_kws_first
                        : (r0 && c->r0_order == 5 ? o_vad_kws
                           : (r0 && c->r0_order == 6 ? o_plain : (r0 ? o_vad : o_plain))));
    for (int i = 0; i < 3; ++i) {
        const int n = order[i];
        void *st = c->serial ? c->stream : c->ns[n];
        const int timed = c->timing && r < MAX_TIMED;
        if (c->fused) {
            if (r == 0) {
                if (c->serial || n != 1) TRY(nnspk_stream_wait(st, c->ev_fork)); /* casc_begin (on VAD's stream) */
            } else {
                for (int m = 0; m < 3; ++m)
                    if (m != n) TRY(nnspk_stream_wait(st, c->ev_rnd[(r - 1) & 1][m]));
            }
        } else if (!c->serial) {
            TRY(nnspk_stream_wait(st, c->ev_fork));
        }
        if (timed) TRY(nnspk_event_record(c->ev_t[r][n][0], st));
        TRY(segment_features(c, n, r, pcm, T, cur, hist, st));
        DBG(st, "cold front end", n, r);
        if (timed) TRY(nnspk_event_record(c->ev_t[r][n][1], st));
        /* S2I's and KWS's round-0 NN waits for VAD's proj; their cold front
         * ends do not (they ran behind VAD's recurrence for CUs, ~85 us, on
         * the round's critical path; A/B 1.010 vs 0.995 G) */
        if (vad_first && n != 1) TRY(nnspk_stream_wait(st, c->ev_vad_proj));
        void *pd = vad_first && n == 1 ? c->ev_vad_proj : (vad_last && n != 1 ? c->ev_r0proj[n] : NULL);
        if (r == 1 && c->fused && !c->serial && c->ahead_mode == 1) pd = c->ev_r1proj[n];
        TRY(round_nn(c, a, r, n, T, cur, hist, st, pd, vad_last && n == 1 ? c->ev_r0proj[0] : NULL,
                     vad_last && n == 1 ? c->ev_r0proj[2] : NULL));
    }
    if (c->fused) return 0;
    return nnspk_launch_casc_control(a, c->stream);
}

/* fused control: the main stream waits for the nets' last launched round */
static int join_rounds(nnsp_cascade *c, int r)
{
    if (!c->fused || r <= 0) return 0;
    for (int n = 0; n < 3; ++n) TRY(nnspk_stream_wait(c->stream, c->ev_rnd[(r - 1) & 1][n]));
    return 0;
}

/* The shared front end of chunk k (log-Mel of every frame into ring slots
 * abs0 .. abs0 + T - 1; the PCM history of chunk k + 1 into d_hist[(k+1) % 3]
 * when T >= H) on the cascade's stream.  tail: the samples of the two frames
 * before the chunk, tail_stride apart per stream. */
static int shared_fe(nnsp_cascade *c, const int16_t *pcm, int T, const int16_t *tail, int tail_stride, int abs0,
                     long long k, int ahead, void *stream)
{
    FeArgs fa;
    memset(&fa, 0, sizeof fa);
    fa.tb_img = c->d_fetab;
    fa.sched = c->fe_sched;
    (void)ahead;
    fa.pcm = pcm;
    fa.tail = tail;
    fa.tail_stride = tail_stride;
    fa.S = c->S;
    fa.T = T;
    fa.mean = c->net[0]->d_mean; /* unused in FE_MODE_SHARED */
    fa.stdR = c->net[0]->d_stdR;
    fa.mode = FE_MODE_SHARED;
    fa.dbg_clk = c->net[1]->d_clk; /* development probe (NNSP_RECUR_CLOCKS): per-wave records in VAD's buffer */
    fa.port = c->net[0]->port;
    fa.norm32 = c->net[0]->norm32 && c->net[1]->norm32 && c->net[2]->norm32;
    fa.ring = c->ring;
    fa.abs0 = abs0;
    for (int n = 0; n < 3; ++n) {
        fa.nring[n] = c->d_nring[n];
        fa.nmean[n] = c->net[n]->d_mean;
        fa.nstdR[n] = c->net[n]->d_stdR;
        fa.nshift[n] = c->net[n]->norm_shift;
    }
    if (T >= c->H) { /* the next chunk's look-back history, stored by the front end */
        fa.hist_out = c->d_hist[(k + 1) % 3];
        fa.hist_frames = c->H;
    }
    return nnspk_launch_fe(&fa, stream);
}

/* The last chunk's bookkeeping: wait for the pinned copy of its counters
 * (long done by the time the host comes back) and derive the host-side
 * statistics and the next chunk's window. */
/* the duration of look-ahead slot q, once its front end has finished (wait:
 * block until it has) */
static int ahead_read(nnsp_cascade *c, int q, int wait)
{
    if (!c->ahead_pending[q]) return 0;
    if (!wait && !nnspk_event_done(c->ev_ahead[q][1])) return 0;
    TRY(nnspk_event_sync(c->ev_ahead[q][1]));
    TRY(nnspk_event_elapsed(&c->ahead_ms[q], c->ev_ahead[q][0], c->ev_ahead[q][1]));
    c->ahead_pending[q] = 0;
    return 0;
}

static int book_take(nnsp_cascade *c)
{
    if (!c->book_pending) return 0;
    TRY(nnspk_event_sync(c->ev_book));
    c->book_pending = 0;
    const char *h = (const char *)c->h_book;   /* d_zero: frames[3], counts[18], last_round, cuts, rcount */
    memcpy(c->book_frames, h, sizeof c->book_frames);
    const int32_t *cnt = (const int32_t *)(h + 3 * 8);
    const int32_t(*rc)[3] = (const int32_t(*)[3])(cnt + 20);
    const int r = c->book_rounds, ahead = c->book_ahead;
    c->last_rounds = cnt[18] + 1;
    c->last_cuts = cnt[19];
    if (c->auto_window) {
        /* window for the next chunk from this chunk's net switches per stream:
         * few switches -> run each stream to the chunk end in one round (a
         * switch then wastes the rest of the chunk's work on that stream, but
         * rounds are few); frequent switches -> short windows bound the waste.
         * Results do not depend on the window (tests/test_gpu_cascade.py). */
        const double per = (double)c->last_cuts / (double)c->S;
        c->window = per < 0.5 ? 0 : (per < 2.0 ? 32 : 16);
    }
    (void)ahead;
    /* the shared front end of that chunk: run in the call (ev_fe), or ahead by
     * the previous call (its slot, once finished; else the last known value) */
    if (!c->book_ahead_done) {
        TRY(nnspk_event_elapsed(&c->sfe_ms, c->ev_fe[0], c->ev_fe[1]));
    } else {
        TRY(ahead_read(c, (int)((c->chunk - 1) & 1), 0));
        c->sfe_ms = c->ahead_ms[(c->chunk - 1) & 1];
    }
    {   /* running totals: read once after a timed loop instead of per chunk */
        float cms = 0.f;
        TRY(nnspk_event_elapsed(&cms, c->ev[0], c->ev[1]));
        c->tot_chunks++;
        c->tot_rounds += c->last_rounds;
        c->tot_frames += c->book_frames[0] + c->book_frames[1] + c->book_frames[2];
        c->tot_fe_ms += c->sfe_ms;
        c->tot_chunk_ms += cms;
    }
    memcpy(c->rc, rc, sizeof c->rc);
    memset(c->rfe, 0, sizeof c->rfe);
    memset(c->rnn, 0, sizeof c->rnn);
    for (int k = r; k < MAX_TIMED; ++k) c->rc[k][0] = c->rc[k][1] = c->rc[k][2] = 0;
    for (int n = 0; n < 3; ++n) {
        c->fe_ms[n] = c->nn_ms[n] = 0.f;
        c->runs[n] = 0;
        for (int k = 0; k < r && k < MAX_TIMED; ++k) {
            if (!c->rc[k][n]) continue;
            c->runs[n]++;
            if (!c->timing) continue;
            float fe = 0.f, nn = 0.f;
            TRY(nnspk_event_elapsed(&fe, c->ev_t[k][n][0], c->ev_t[k][n][1]));
            TRY(nnspk_event_elapsed(&nn, c->ev_t[k][n][1], c->ev_t[k][n][2]));
            c->fe_ms[n] += fe;
            c->nn_ms[n] += nn;
            c->rfe[k][n] = fe;
            c->rnn[k][n] = nn;
        }
    }
    return 0;
}

int nnsp_cascade_exec_device(nnsp_cascade *c, const int16_t *pcm, int T, int8_t *net_ran, int16_t *detected,
                             int16_t *outputs3)
{
    return nnsp_cascade_exec_device_ahead(c, pcm, T, NULL, 0, net_ran, detected, outputs3);
}

int nnsp_cascade_exec_device_ahead(nnsp_cascade *c, const int16_t *pcm, int T, const int16_t *next_pcm, int next_T,
                                   int8_t *net_ran, int16_t *detected, int16_t *outputs3)
{
    if (!c || !pcm || T <= 0 || T > c->Tmax || (next_pcm && (next_T <= 0 || next_T > c->Tmax))) {
        nnsp_set_error("nnsp_cascade_exec: T must be in 1..%d", c ? c->Tmax : 0);
        return NNSP_EINVAL;
    }
    TRY(book_take(c)); /* the last chunk's counters: rounds, switches (this chunk's window) */
    const long long k = c->chunk;
    zero_bind(c, (int)(k & 1));
    if (c->chunk_open) /* the last call failed after launching rounds into this block */
        TRY(nnspk_memset((char *)c->d_zero + (size_t)(k & 1) * ZERO_STRIDE, 0, ZERO_BYTES, c->stream));
    c->chunk_open = 1;
    CascArgs a = c->a;
    a.T = T;
    a.seg_len = c->window;
    a.net_ran = net_ran;
    a.detected = detected;
    a.outputs3 = outputs3;
    for (int n = 0; n < 3; ++n) a.fs[n].abs0 = c->abs0;
    /* look-ahead: the next chunk's shared front end runs while this chunk's
     * rounds run (it writes ring slots and a history buffer this chunk does not
     * read; its STFT tail is this chunk's last two frames) */
    const int ahead = next_pcm && T >= 2 && T >= c->H && next_T >= c->H && c->fused && !c->serial;
    /* 1. log-Mel of every frame (net-independent), unless the previous call ran it ahead */
    const int ahead_done = c->pre_pcm == pcm && c->pre_T == T;
    c->pre_pcm = NULL;
    if (!ahead_done) {   /* (the chunk's start: ev[0]; ran ahead, casc_begin is launched first) */
        TRY(nnspk_event_record(c->ev[0], c->stream));
        TRY(nnspk_event_record(c->ev_fe[0], c->stream));
        TRY(shared_fe(c, pcm, T, c->d_stail, 0, c->abs0, k, 0, c->stream));
        DBG(c->stream, "shared front end", -1, -1);
        TRY(nnspk_event_record(c->ev_fe[1], c->stream));
    }
    c->sfe_ahead = ahead_done;
    const int16_t *hist = c->d_hist[k % 3];
    a.counts = c->d_counts; /* round 0's lists */
    for (int n = 0; n < 3; ++n) {
        a.list[n] = c->d_list[0][n];
        a.cold_list[n] = c->d_cold_list[0][n];
    }
    /* fused control: casc_begin on VAD's stream, which runs round 0 first --
     * VAD's cold front end then follows it in order instead of behind a
     * cross-queue event wait (~12 us); it waits only for a front end this
     * call ran itself (in the steady state the previous call ran it ahead) */
    const int begin_on_vad = c->fused && !c->serial;
    void *bst = begin_on_vad ? c->ns[1] : c->stream;
    if (begin_on_vad && !ahead_done) TRY(nnspk_stream_wait(bst, c->ev_fe[1]));
    /* early return: the previous call returned before the look-ahead front end
     * of this chunk had finished -- round 0 waits for it on the device */
    if (ahead_done && c->early_prev) TRY(nnspk_stream_wait(bst, c->ev_ahead[k & 1][1]));
    TRY(nnspk_launch_casc_begin(&a, bst));
    DBG(bst, "casc_begin", -1, -1);
    /* c->stream is idle: about now -- except after an early return, when the
     * look-ahead front end may still run on it: ev[0] then goes on bst, behind
     * the wait for that front end, so that it completes before ev[1] (on the
     * book stream) and book_take's elapsed time is always ready */
    if (ahead_done) TRY(nnspk_event_record(c->ev[0], c->early_prev ? bst : c->stream));
    if (c->fused) TRY(nnspk_event_record(c->ev_fork, bst));
    int ahead_launched = 0, behind_launched = 0;
    /* the look-ahead front end starts once the nets' first round (the bulk of
     * the chunk's NN work) is done: running beside it from the start, or with
     * its workgroups capped or short-lived, or on a CU partition, it slowed
     * the rounds more than it gained (profiles/r02/sched; round 3, persistent
     * and CU-masked variants: profiles/r03/cofe/README.md); started once VAD's
     * round 0 is done and S2I's and KWS's recurrences are queued: 0.975 vs
     * 0.992 G (4 paired runs) */
    /* rounds launched before the first host check: as many as the last chunk
     * needed, at least 3 (the reference nets' usual count: a chunk that needs
     * one more than launched pays a host round trip, ~80 us, an empty round
     * launched in vain a few us of early-exiting workgroups) */
    int r = 0, R = c->last_rounds > 0 ? (c->last_rounds < 3 ? 3 : c->last_rounds) : 8;
    for (;;) {
        for (; r < R; ++r) {
            TRY(launch_round(c, &a, r, pcm, T, hist));
            if (!behind_launched) {
                /* behind the fork, launched after round 0 (the GPU waited ~30 us
                 * for round 0's first kernel while the host enqueued these ahead
                 * of it): nothing in this chunk reads what they write -- the
                 * cold frames read d_hist[k % 3], the look-ahead front end takes
                 * its tail from pcm */
                if (T < c->H) /* shorter chunk: part of the history comes from the previous one */
                    TRY(nnspk_launch_hist_roll(c->d_hist[(k + 1) % 3], hist, pcm, c->S, T, c->H, c->stream));
                TRY(nnspk_launch_tail_roll(c->d_stail, pcm, c->S, T, NULL, 0, NULL, 0, 0, NULL, 0, c->stream));
                /* the next chunk's counters (copied out and taken at the end of the last call) */
                TRY(nnspk_memset((char *)c->d_zero + (size_t)((k + 1) & 1) * ZERO_STRIDE, 0, ZERO_BYTES, c->stream));
                behind_launched = 1;
            }
            /* ahead_mode (NNSP_AHEAD_MODE): 0 the front end waits for round 0's
             * end; 1 (default) for round 1's proj, so that round 1's proj runs
             * on an idle device and its recurrences are on the CUs before the
             * front end's workgroups flood them -- before, they waited for the
             * front end to drain and ran after it (~190 us past its end);
             * 2 for round 1's end.  A/B 1.099 / 1.149 / 1.111 G (modes 0 / 1
             * / 2, 2 runs each), profiles/r04/ahead_mode/ */
            /* (ahead implies fused && !serial: the only mode in which round 1
             * records ev_r1proj and every round records ev_rnd) */
            const int am = c->fused && !c->serial ? c->ahead_mode : 0;
            if (ahead && !ahead_launched && r >= (am ? 1 : 0)) {
                for (int n = 0; n < 3; ++n)
                    TRY(nnspk_stream_wait(c->stream, am == 1 ? c->ev_r1proj[n] : c->ev_rnd[r & 1][n]));
                const int q = (int)((k + 1) & 1);
                TRY(ahead_read(c, q, 1)); /* slot q's last front end (two chunks ago) is long done */
                TRY(nnspk_event_record(c->ev_ahead[q][0], c->stream));
                TRY(shared_fe(c, next_pcm, next_T, pcm + (size_t)(T - 2) * 160, T * 160, (c->abs0 + T) % c->ring,
                              k + 1, 1, c->stream));
                TRY(nnspk_event_record(c->ev_ahead[q][1], c->stream));
                c->ahead_pending[q] = 1;
                ahead_launched = 1;
            }
        }
        /* early return (with a look-ahead front end running on c->stream): the
         * join and the counter copy on the book stream, so that they do not
         * queue behind the front end */
        const int er = c->early && ahead_launched;
        void *js = er ? c->bstream : c->stream;
        if (er) {
            for (int n = 0; n < 3; ++n) TRY(nnspk_stream_wait(js, c->ev_rnd[(r - 1) & 1][n]));
        } else {
            TRY(join_rounds(c, r));
        }
        TRY(nnspk_event_record(c->ev[1], js)); /* the rounds' end (complete at the sync below) */
        /* all the chunk's counters in one copy (the next round's list lengths
         * among them): if no round is left they are final, and the
         * bookkeeping needs no further host wait */
        TRY(nnspk_d2h(c->h_book, c->d_frames, ZERO_BYTES, js));
        TRY(nnspk_event_record(c->ev_book, js));
        /* polled, not a blocking stream synchronisation: the wake-up of a
         * blocking wait sits between this chunk's last kernel and the next
         * chunk's first (everything on c->stream is before ev_book); the
         * host first sleeps through the look-ahead front end, so it polls
         * only through the rounds' tail (A/B: 1.004 vs 0.997 G) */
        /* without a look-ahead front end to sleep through, the whole chunk is
         * still ahead: a blocking wait, not a core spinning for milliseconds */
        if (er) {   /* the rounds' end, not the front end's: polled */
            TRY(nnspk_event_spin(c->ev_book));
        } else if (ahead_launched) {
            TRY(nnspk_event_sync(c->ev_ahead[(k + 1) & 1][1]));
            TRY(nnspk_event_spin(c->ev_book));
        } else {
            TRY(nnspk_event_sync(c->ev_book));
        }
        const int32_t *cnt = (const int32_t *)((const char *)c->h_book + 3 * 8) + 6 * (r % 3);
        if (cnt[0] + cnt[1] + cnt[2] == 0) break;
        R = r + 2;
    }
    c->launched = r;
    c->chunk_open = 0;
    c->early_prev = c->early && ahead_launched;
    c->abs0 = (c->abs0 + T) % c->ring;
    c->chunk = k + 1;
    if (ahead_launched) {
        c->pre_pcm = next_pcm;
        c->pre_T = next_T;
    }
    /* bookkeeping: h_book was copied before the last synchronisation, so it
     * is taken now (no host wait at the next call); this parity's device
     * counters are cleared by the chunk after next, behind its fork */
    c->book_pending = 1;
    c->book_rounds = r;
    c->book_ahead = ahead_launched;
    c->book_ahead_done = ahead_done;
    TRY(book_take(c));
    return 0;
}

static int ensure(void **p, size_t bytes)
{
    if (*p) return 0;
    return nnspk_malloc(p, bytes);
}

int nnsp_cascade_exec(nnsp_cascade *c, const int16_t *pcm, int T, int8_t *net_ran, int16_t *detected,
                      int16_t *outputs3)
{
    if (!c || !pcm || T <= 0 || T > c->Tmax) return NNSP_EINVAL;
    const size_t S = (size_t)c->S, TT = (size_t)c->Tmax;
    TRY(ensure((void **)&c->d_pcm, S * TT * 320));
    if (net_ran) TRY(ensure((void **)&c->d_ran, S * TT));
    if (detected) TRY(ensure((void **)&c->d_det, S * TT * 2));
    if (outputs3) TRY(ensure((void **)&c->d_o3, S * TT * 6));
    TRY(nnspk_h2d(c->d_pcm, pcm, S * T * 320, c->stream));
    TRY(nnsp_cascade_exec_device(c, c->d_pcm, T, net_ran ? c->d_ran : NULL, detected ? c->d_det : NULL,
                                 outputs3 ? c->d_o3 : NULL));
    if (net_ran) TRY(nnspk_d2h(net_ran, c->d_ran, S * T, c->stream));
    if (detected) TRY(nnspk_d2h(detected, c->d_det, S * T * 2, c->stream));
    if (outputs3) TRY(nnspk_d2h(outputs3, c->d_o3, S * T * 6, c->stream));
    return nnspk_sync(c->stream);
}

int nnsp_cascade_set_window(nnsp_cascade *c, int frames)
{
    if (!c || frames < -1) return NNSP_EINVAL;
    c->auto_window = frames < 0;
    if (frames >= 0) c->window = frames;
    return 0;
}

int nnsp_cascade_get_window(nnsp_cascade *c, int *frames, int *is_auto, int *last_cuts)
{
    if (!c) return NNSP_EINVAL;
    TRY(book_take(c));
    if (frames) *frames = c->window;
    if (is_auto) *is_auto = c->auto_window;
    if (last_cuts) *last_cuts = c->last_cuts;
    return 0;
}

int nnsp_cascade_set_timing(nnsp_cascade *c, int on)
{
    if (!c) return NNSP_EINVAL;
    c->timing = on != 0;
    return 0;
}

int nnsp_cascade_set_serial(nnsp_cascade *c, int on)
{
    if (!c) return NNSP_EINVAL;
    TRY(nnspk_sync(c->stream));
    c->serial = on != 0;
    return 0;
}

int nnsp_cascade_sync(nnsp_cascade *c)
{
    if (!c) return NNSP_EINVAL;
    TRY(nnspk_sync(c->stream));
    if (c->bstream) TRY(nnspk_sync(c->bstream));
    TRY(book_take(c));
    for (int q = 0; q < 2; ++q) TRY(ahead_read(c, q, 1));
    return 0;
}
void *nnsp_cascade_stream(nnsp_cascade *c) { return c ? c->stream : NULL; }

int nnsp_cascade_last_stats(nnsp_cascade *c, int *rounds, long long *frames_run, float *ms)
{
    if (!c) return NNSP_EINVAL;
    TRY(book_take(c));
    if (rounds) *rounds = c->last_rounds;
    if (frames_run) *frames_run = (long long)(c->book_frames[0] + c->book_frames[1] + c->book_frames[2]);
    if (ms) TRY(nnspk_event_elapsed(ms, c->ev[0], c->ev[1]));
    return 0;
}

int nnsp_cascade_last_fe_stats(nnsp_cascade *c, float *ms)
{
    if (!c) return NNSP_EINVAL;
    TRY(book_take(c));
    if (ms) *ms = c->sfe_ms;
    return 0;
}

int nnsp_cascade_last_net_stats(nnsp_cascade *c, int nn_id, long long *frames_run, float *fe_ms, float *nn_ms,
                                int *launches)
{
    if (!c || nn_id < 0 || nn_id > 2) return NNSP_EINVAL;
    TRY(book_take(c));
    if (frames_run) *frames_run = (long long)c->book_frames[nn_id];
    if (fe_ms) *fe_ms = c->fe_ms[nn_id];
    if (nn_ms) *nn_ms = c->nn_ms[nn_id];
    if (launches) *launches = c->runs[nn_id];
    return 0;
}

int nnsp_cascade_last_rounds(nnsp_cascade *c, int max_rounds, int32_t *lists, float *fe_ms, float *nn_ms)
{
    if (!c || max_rounds < 0) return NNSP_EINVAL;
    TRY(book_take(c));
    const int n = c->launched < MAX_TIMED ? c->launched : MAX_TIMED;
    for (int k = 0; k < max_rounds && k < n; ++k)
        for (int i = 0; i < 3; ++i) {
            if (lists) lists[3 * k + i] = c->rc[k][i];
            if (fe_ms) fe_ms[3 * k + i] = c->rfe[k][i];
            if (nn_ms) nn_ms[3 * k + i] = c->rnn[k][i];
        }
    return n;
}

int nnsp_cascade_positions(nnsp_cascade *c, int8_t *pos)
{
    if (!c || !pos) return NNSP_EINVAL;
    CascState *h = (CascState *)malloc((size_t)c->S * sizeof(CascState));
    if (!h) return NNSP_ENOMEM;
    int e = nnspk_d2h(h, c->d_st, (size_t)c->S * sizeof(CascState), c->stream);
    if (!e) e = nnspk_sync(c->stream);
    if (!e)
        for (int s = 0; s < c->S; ++s) pos[s] = (int8_t)h[s].pos;
    free(h);
    return e;
}

/* ---- per-stream state export / import (include/nnsp_cascade.h) ---- */
_Static_assert(sizeof(nnsp_cascade_stream_hdr) == 32, "nnsp_cascade_stream_hdr: 32 bytes");
_Static_assert(sizeof(CascState) == 8, "CascState: the header's 8 bytes at offset 8");

size_t nnsp_cascade_state_bytes(const nnsp_cascade *c)
{
    if (!c) return 0;
    size_t n = sizeof(nnsp_cascade_stream_hdr) + (size_t)c->H * 320 + 640 + 3 * (size_t)(c->H - 2) * 80;
    for (int i = 0; i < 3; ++i) n += nnsp_batch_state_bytes(c->net[i]);
    return n;
}

/* the segments of a stream's blob; valid between chunks (after any work) */
static void cascade_state_segs(const nnsp_cascade *c, StateCopy *sc)
{
    const size_t H = (size_t)c->H;
    size_t off = 0;
    int k = 0;
    StateSeg *g = sc->seg;
    memset(g, 0, sizeof sc->seg);
    /* controller state at header offset 8 (CascState: pos, cnt_kws, cnt_s2i, pad) and frames since the reset at 16 */
    g[k++] = (StateSeg){(unsigned long long)(uintptr_t)c->d_st, sizeof(CascState), 0, 1, sizeof(CascState), 0, 1, 8, 0};
    g[k++] = (StateSeg){(unsigned long long)(uintptr_t)c->d_fresh, 1, 0, 1, 1, 0, 1, 16, 0};
    off = sizeof(nnsp_cascade_stream_hdr);
    /* the history the next chunk reads: d_hist[chunk % 3] */
    g[k++] = (StateSeg){(unsigned long long)(uintptr_t)c->d_hist[c->chunk % 3], H * 320, 0, 1, (uint32_t)(H * 320), 0, 1,
                        (uint32_t)off, 0};
    off += H * 320;
    g[k++] = (StateSeg){(unsigned long long)(uintptr_t)c->d_stail, 640, 0, 1, 640, 0, 1, (uint32_t)off, 0};
    off += 640;
    /* ring slots abs0 - (H - 2) .. abs0 - 1 (the look-back frames: a net at
     * look-back L reads frames -L .. -1 of them), oldest first */
    for (int n = 0; n < 3; ++n) {
        if (H > 2)
            g[k++] = (StateSeg){(unsigned long long)(uintptr_t)c->d_nring[n], (unsigned long long)c->ring * 80, 80,
                                (uint32_t)(H - 2), 80, (uint32_t)((c->abs0 - (int)(H - 2) + c->ring) % c->ring),
                                (uint32_t)c->ring, (uint32_t)off, 0};
        off += (H - 2) * 80;
    }
    for (int n = 0; n < 3; ++n) k += nnsp_batch_state_segs(c->net[n], g + k, off, &off);
    sc->nseg = k;
    sc->per = off;
}

/* the nets' state shapes, as set_state must find them (a blob of other nets
 * of the same size would otherwise be imported silently) */
static uint32_t cascade_nets_sig(const nnsp_cascade *c)
{
    uint32_t h = 2166136261u;
    for (int n = 0; n < 3; ++n) {
        const nnsp_batch *b = c->net[n];
        const uint32_t v[4] = {(uint32_t)b->hs, (uint32_t)b->im.img.n_lstm, (uint32_t)b->nout,
                               (uint32_t)nnsp_batch_state_bytes(b)};
        for (int i = 0; i < 4; ++i)
            for (int k = 0; k < 4; ++k) h = (h ^ ((v[i] >> (8 * k)) & 0xffu)) * 16777619u;
    }
    return h;
}

static int cascade_quiesce(nnsp_cascade *c)
{
    TRY(nnspk_sync(c->stream));
    if (c->bstream) TRY(nnspk_sync(c->bstream));
    for (int n = 0; n < 3; ++n) TRY(nnspk_sync(c->ns[n]));
    TRY(book_take(c));
    for (int q = 0; q < 2; ++q) TRY(ahead_read(c, q, 1));
    return 0;
}

int nnsp_cascade_get_state(nnsp_cascade *c, void *host, int first, int count)
{
    if (!c || !host || first < 0 || count < 0 || first + count > c->S) return NNSP_EINVAL;
    TRY(cascade_quiesce(c));
    StateCopy sc;
    memset(&sc, 0, sizeof sc);
    cascade_state_segs(c, &sc);
    sc.first = first;
    sc.count = count;
    sc.to_blob = 1;
    memset(host, 0, (size_t)count * sc.per);
    TRY(nnsp_state_xfer(&sc, host, c->stream));
    for (int i = 0; i < count; ++i) {
        nnsp_cascade_stream_hdr *h = (nnsp_cascade_stream_hdr *)((char *)host + (size_t)i * sc.per);
        h->magic = NNSP_CASCADE_STATE_MAGIC;
        h->hist_frames = (uint16_t)c->H;
        h->version = NNSP_CASCADE_STATE_VERSION;
        h->state_bytes = (uint32_t)sc.per;
        h->nets_sig = cascade_nets_sig(c);
    }
    return 0;
}

int nnsp_cascade_set_state(nnsp_cascade *c, const void *host, int first, int count)
{
    if (!c || !host || first < 0 || count < 0 || first + count > c->S) return NNSP_EINVAL;
    StateCopy sc;
    memset(&sc, 0, sizeof sc);
    cascade_state_segs(c, &sc);
    const uint32_t sig = cascade_nets_sig(c);
    for (int i = 0; i < count; ++i) {
        const nnsp_cascade_stream_hdr *h = (const nnsp_cascade_stream_hdr *)((const char *)host + (size_t)i * sc.per);
        if (h->magic != NNSP_CASCADE_STATE_MAGIC || h->version != NNSP_CASCADE_STATE_VERSION) {
            nnsp_set_error("nnsp_cascade_set_state: blob %d is not a cascade stream state (version %d)", i,
                           NNSP_CASCADE_STATE_VERSION);
            return NNSP_EINVAL;
        }
        if (h->hist_frames != c->H || h->state_bytes != (uint32_t)sc.per || h->nets_sig != sig) {
            nnsp_set_error("nnsp_cascade_set_state: blob %d is the state of another cascade (%u history frames, "
                           "%u bytes, nets %08x; this one: %d, %zu, %08x)", i, (unsigned)h->hist_frames,
                           (unsigned)h->state_bytes, (unsigned)h->nets_sig, c->H, sc.per, (unsigned)sig);
            return NNSP_EINVAL;
        }
    }
    TRY(cascade_quiesce(c));
    cascade_state_segs(c, &sc);
    sc.first = first;
    sc.count = count;
    sc.to_blob = 0;
    TRY(nnsp_state_xfer(&sc, (void *)host, c->stream));
    c->pre_pcm = NULL; /* a look-ahead front end ran on the old state: the next call recomputes */
    return 0;
}

/* ---- the reference's per-stream objects (include/nnsp_cascade.h) ----
 * A blob (nnsp_cascade_get_state's layout) is built from / taken apart into
 * the objects the reference keeps per stream: nnCntrlClass
 * (evb/src/nnCntrlClass.h:35-45), PcmBufClass (PcmBufClass.c:10-85), and per
 * net NNSPClass (nn_speech.h:12-25), FeatureClass (feature_module.h:7-18) and
 * the LSTM state of its NeuralNetClass.  Only the layout moves here; the
 * look-back features, which the reference does not keep, are recomputed on
 * the device by the shared front end. */
typedef struct {
    size_t hist, stail, look, net[3];
} blob_offs;

static blob_offs blob_layout(const nnsp_cascade *c)
{
    blob_offs o;
    o.hist = sizeof(nnsp_cascade_stream_hdr);
    o.stail = o.hist + (size_t)c->H * 320;
    o.look = o.stail + 640;
    o.net[0] = o.look + 3 * (size_t)(c->H - 2) * 80;
    o.net[1] = o.net[0] + nnsp_batch_state_bytes(c->net[0]);
    o.net[2] = o.net[1] + nnsp_batch_state_bytes(c->net[1]);
    return o;
}

/* frame -j (j >= 1, 1 = the newest) of the voice buffer (PcmBufClass_getData
 * with lookbk_frs = j - 1), NULL past the frames it holds */
static const int16_t *vbuf_frame(const nnsp_ref_pcmbuf *pb, int j)
{
    if (j < 1 || j > pb->num_frs) return NULL;
    int slot = (pb->idx_data_latest - (j - 1)) % pb->num_frs;
    if (slot < 0) slot += pb->num_frs;
    return pb->pcm_buffer + (size_t)slot * 160;
}

static int all_zero(const int16_t *x, int n)
{
    for (int i = 0; i < n; ++i)
        if (x[i]) return 0;
    return 1;
}

/* the LSTM layers of a reference NeuralNetClass, checked against net n of the
 * cascade (one state row per LSTM layer, hs elements apart in the blob) */
static int ref_lstm_layers(const nnsp_cascade *c, int n, const NeuralNetClass *net, int *layer)
{
    const nnsp_batch *b = c->net[n];
    int k = 0;
    for (int i = 0; i < net->numlayers && i < NN_MAX_LAYERS; ++i)
        if (net->net_layer_type[i] == lstm) {
            if (k >= b->im.img.n_lstm || net->size_layer[i + 1] != b->im.img.lstm_n[k] || !net->pt_hstate[i] ||
                !net->pt_cstate[i])
                return -1;
            layer[k++] = i;
        }
    return k == b->im.img.n_lstm ? k : -1;
}

static void ref_post_pack(const NNSPClass *p, NnPost *q)
{
    memset(q, 0, sizeof *q);
    q->slides = p->slides;
    q->trigger = p->trigger;
    q->argmax_last = p->argmax_last;
    memcpy(q->counts, p->counts_category, sizeof q->counts);
    memcpy(q->outputs, p->outputs, sizeof q->outputs);
}

static void ref_post_unpack(NNSPClass *p, const NnPost *q)
{
    p->slides = (int8_t)q->slides;
    p->trigger = q->trigger;
    p->argmax_last = q->argmax_last;
    memcpy(p->counts_category, q->counts, sizeof q->counts);
    memcpy(p->outputs, q->outputs, sizeof q->outputs);
}

static int ref_check(const nnsp_cascade *c, const nnsp_ref_stream *R, int i, int need_frames)
{
    if (!R->cntrl || !R->pcmbuf || !R->pcmbuf->pcm_buffer) {
        nnsp_set_error("nnsp_cascade state_ref: stream %d: NULL controller or voice buffer", i);
        return NNSP_EINVAL;
    }
    const nnsp_ref_pcmbuf *pb = R->pcmbuf;
    if (pb->smpls_fr != 160 || pb->num_frs < need_frames || pb->idx_data_latest < 0 ||
        pb->idx_data_latest >= pb->num_frs) {
        nnsp_set_error("nnsp_cascade state_ref: stream %d: voice buffer of %d x %d samples (latest %d); 160-sample "
                       "frames, at least %d of them, are needed", i, pb->num_frs, pb->smpls_fr, pb->idx_data_latest,
                       need_frames);
        return NNSP_EINVAL;
    }
    if (R->cntrl->len_seq_cntrl != c->len_seq || R->cntrl->current_pos_seq < 0 ||
        R->cntrl->current_pos_seq >= c->len_seq) {
        nnsp_set_error("nnsp_cascade state_ref: stream %d: position %d of a sequence of %d (the cascade's: %d)", i,
                       R->cntrl->current_pos_seq, R->cntrl->len_seq_cntrl, c->len_seq);
        return NNSP_EINVAL;
    }
    for (int n = 0; n < 3; ++n) {
        const NNSPClass *q = R->nnsp[n];
        int layer[NN_MAX_LSTM];
        if (!q || (int)q->nn_id != n || !q->pt_feat || !q->pt_net ||
            ref_lstm_layers(c, n, (const NeuralNetClass *)q->pt_net, layer) < 0) {
            nnsp_set_error("nnsp_cascade state_ref: stream %d: nnsp[%d] is not an NNSPClass of NNSP_ID %d whose net's "
                           "LSTM layers are the cascade's", i, n, n);
            return NNSP_EINVAL;
        }
    }
    return 0;
}

int nnsp_cascade_set_state_ref(nnsp_cascade *c, int first, int count, const nnsp_ref_stream *refs)
{
    if (!c || !refs || first < 0 || count < 0 || first + count > c->S) return NNSP_EINVAL;
    if (count == 0) return 0;
    const size_t per = nnsp_cascade_state_bytes(c);
    const blob_offs o = blob_layout(c);
    const int H = c->H;
    const uint32_t sig = cascade_nets_sig(c);
    uint8_t *blob = (uint8_t *)calloc((size_t)count, per);
    if (!blob) return NNSP_ENOMEM;
    int e = 0;
    for (int i = 0; i < count && !e; ++i) {
        const nnsp_ref_stream *R = &refs[i];
        /* frames -(H-1) .. -1: the look-back frame of every net and the one
         * before it; frame -H only as the STFT buffer's oldest frame */
        if ((e = ref_check(c, R, i, H - 1))) break;
        uint8_t *b = blob + (size_t)i * per;
        nnsp_cascade_stream_hdr *h = (nnsp_cascade_stream_hdr *)b;
        h->magic = NNSP_CASCADE_STATE_MAGIC;
        h->hist_frames = (uint16_t)H;
        h->version = NNSP_CASCADE_STATE_VERSION;
        h->state_bytes = (uint32_t)per;
        h->nets_sig = sig;
        h->current_pos_seq = R->cntrl->current_pos_seq;
        h->cnt_timeout_kws = R->cntrl->cnt_timeout_kws;
        h->cnt_timeout_s2i = R->cntrl->cnt_timeout_s2i;
        const nnsp_ref_pcmbuf *pb = R->pcmbuf;
        int16_t *hist = (int16_t *)(b + o.hist);   /* [H][160], frame -H first */
        for (int j = 1; j <= H; ++j) {
            const int16_t *f = vbuf_frame(pb, j);
            if (f) memcpy(hist + (size_t)(H - j) * 160, f, 320);
        }
        memcpy(b + o.stail, hist + (size_t)(H - 2) * 160, 640);
        /* the net at the current position: frames since its reset, from its
         * STFT buffer (dataBuffer[160..479] = the two frames before its next
         * one; zero before a reset, stftModule_setDefault); the other two are
         * reset when the controller leaves them */
        const int cur = c->seq[R->cntrl->current_pos_seq], L = c->lookback[cur];
        int fresh = -1;
        for (int n = 0; n < 3 && !e; ++n) {
            const FeatureClass *fe = (const FeatureClass *)R->nnsp[n]->pt_feat;
            const int16_t *A = fe->state_stftModule.dataBuffer + 160, *B = A + 160;
            if (n != cur) {
                if (!all_zero(A, 320)) {
                    nnsp_set_error("nnsp_cascade_set_state_ref: stream %d: net %d is not at the current position "
                                   "and its STFT buffer is not reset", i, n);
                    e = NNSP_EINVAL;
                }
                continue;
            }
            const int16_t *F1 = vbuf_frame(pb, L + 1), *F2 = vbuf_frame(pb, L + 2);
            /* (where two readings fit -- zero frames in the voice buffer --
             * both give the same outputs) */
            if (!memcmp(B, F1, 320) && F2 && !memcmp(A, F2, 320)) {
                fresh = 2;
            } else if (all_zero(A, 160) && !memcmp(B, F1, 320)) {
                fresh = 1;
            } else if (!F2 && !memcmp(B, F1, 320)) {
                fresh = 2;
                memcpy(hist, A, 320);   /* frame -(L + 2) = -H: past the voice buffer */
            } else if (all_zero(A, 320)) {
                fresh = 0;
            } else {
                nnsp_set_error("nnsp_cascade_set_state_ref: stream %d: the STFT buffer of net %d does not hold the "
                               "voice buffer's frames at look-back %d", i, n, L);
                e = NNSP_EINVAL;
            }
        }
        if (e) break;
        h->frames_since_reset = (int8_t)fresh;
        for (int n = 0; n < 3; ++n) {
            const nnsp_batch *nb = c->net[n];
            const NNSPClass *q = R->nnsp[n];
            const FeatureClass *fe = (const FeatureClass *)q->pt_feat;
            const NeuralNetClass *net = (const NeuralNetClass *)q->pt_net;
            uint8_t *nbp = b + o.net[n];   /* [STFT tail 640, unused by the cascade: 0][prev5 400][h][c][post] */
            memcpy(nbp + 640, fe->normFeatContext + 40, 400);
            int layer[NN_MAX_LSTM];
            const int nl = ref_lstm_layers(c, n, net, layer);
            const size_t hb = (size_t)(nl ? nl : 1) * nb->hs * 2;
            for (int l = 0; l < nl; ++l) {
                const int N = net->size_layer[layer[l] + 1];
                memcpy(nbp + 1040 + (size_t)l * nb->hs * 2, net->pt_hstate[layer[l]], (size_t)N * 2);
                memcpy(nbp + 1040 + hb + (size_t)l * nb->hs * 4, net->pt_cstate[layer[l]], (size_t)N * 4);
            }
            NnPost ps;
            ref_post_pack(q, &ps);
            memcpy(nbp + 1040 + hb + hb * 2, &ps, sizeof ps);
        }
    }
    if (!e) e = nnsp_cascade_set_state(c, blob, first, count);
    free(blob);
    if (e) return e;
    /* the look-back features: the shared front end over the imported history
     * (frames -H .. -1 of these streams as a chunk of H frames, written to ring
     * slots abs0 - H .. abs0 - 1).  Frames -H and -(H-1) see a zero STFT tail;
     * no net reads them (a net at look-back L reads frames -L .. -1 of the
     * ring, and L <= H - 2) */
    void *ztail = NULL;
    TRY(nnspk_malloc(&ztail, (size_t)count * 640));
    FeArgs fa;
    memset(&fa, 0, sizeof fa);
    fa.tb_img = c->d_fetab;
    fa.sched = c->fe_sched;
    fa.pcm = c->d_hist[c->chunk % 3] + (size_t)first * H * 160;
    fa.tail = (const int16_t *)ztail;
    fa.S = count;
    fa.T = H;
    fa.mean = c->net[0]->d_mean;
    fa.stdR = c->net[0]->d_stdR;
    fa.mode = FE_MODE_SHARED;
    fa.port = c->net[0]->port;
    fa.norm32 = c->net[0]->norm32 && c->net[1]->norm32 && c->net[2]->norm32;
    fa.ring = c->ring;
    fa.abs0 = (c->abs0 - H + c->ring) % c->ring;
    for (int n = 0; n < 3; ++n) {
        fa.nring[n] = c->d_nring[n] + (size_t)first * c->ring * 40;
        fa.nmean[n] = c->net[n]->d_mean;
        fa.nstdR[n] = c->net[n]->d_stdR;
        fa.nshift[n] = c->net[n]->norm_shift;
    }
    e = nnspk_memset(ztail, 0, (size_t)count * 640, c->stream);
    if (!e) e = nnspk_launch_fe(&fa, c->stream);
    if (!e) e = nnspk_sync(c->stream);
    nnspk_free(ztail);
    return e;
}

int nnsp_cascade_get_state_ref(nnsp_cascade *c, int first, int count, const nnsp_ref_stream *refs)
{
    if (!c || !refs || first < 0 || count < 0 || first + count > c->S) return NNSP_EINVAL;
    if (count == 0) return 0;
    const int H = c->H;
    for (int i = 0; i < count; ++i) TRY(ref_check(c, &refs[i], i, H - 1));
    const size_t per = nnsp_cascade_state_bytes(c);
    const blob_offs o = blob_layout(c);
    uint8_t *blob = (uint8_t *)malloc((size_t)count * per);
    if (!blob) return NNSP_ENOMEM;
    int e = nnsp_cascade_get_state(c, blob, first, count);
    for (int i = 0; i < count && !e; ++i) {
        const nnsp_ref_stream *R = &refs[i];
        const uint8_t *b = blob + (size_t)i * per;
        const nnsp_cascade_stream_hdr *h = (const nnsp_cascade_stream_hdr *)b;
        R->cntrl->current_pos_seq = (int8_t)h->current_pos_seq;
        R->cntrl->cnt_timeout_kws = h->cnt_timeout_kws;
        R->cntrl->cnt_timeout_s2i = h->cnt_timeout_s2i;
        nnsp_ref_pcmbuf *pb = R->pcmbuf;
        const int16_t *hist = (const int16_t *)(b + o.hist);   /* frame -H first */
        memset(pb->pcm_buffer, 0, (size_t)pb->num_frs * 320);
        pb->idx_data_latest = (int16_t)(pb->num_frs - 1);
        pb->idx_set = 0;
        for (int j = 1; j <= H && j <= pb->num_frs; ++j)
            memcpy(pb->pcm_buffer + (size_t)(pb->num_frs - j) * 160, hist + (size_t)(H - j) * 160, 320);
        const int cur = c->seq[h->current_pos_seq], L = c->lookback[cur], fresh = h->frames_since_reset;
        for (int n = 0; n < 3; ++n) {
            const nnsp_batch *nb = c->net[n];
            NNSPClass *q = R->nnsp[n];
            FeatureClass *fe = (FeatureClass *)q->pt_feat;
            NeuralNetClass *net = (NeuralNetClass *)q->pt_net;
            const uint8_t *nbp = b + o.net[n];
            int16_t *db = fe->state_stftModule.dataBuffer;
            memset(db, 0, 480 * 2);
            if (n == cur && fresh >= 1) {   /* [160..319] frame -(L+2), [320..479] frame -(L+1) */
                memcpy(db + 320, hist + (size_t)(H - (L + 1)) * 160, 320);
                if (fresh >= 2) memcpy(db + 160, hist + (size_t)(H - (L + 2)) * 160, 320);
            }
            memset(fe->normFeatContext, 0, 80);
            memcpy(fe->normFeatContext + 40, nbp + 640, 400);
            int layer[NN_MAX_LSTM];
            const int nl = ref_lstm_layers(c, n, net, layer);
            const size_t hb = (size_t)(nl ? nl : 1) * nb->hs * 2;
            for (int l = 0; l < nl; ++l) {
                const int N = net->size_layer[layer[l] + 1];
                memcpy(net->pt_hstate[layer[l]], nbp + 1040 + (size_t)l * nb->hs * 2, (size_t)N * 2);
                memcpy(net->pt_cstate[layer[l]], nbp + 1040 + hb + (size_t)l * nb->hs * 4, (size_t)N * 4);
            }
            NnPost ps;
            memcpy(&ps, nbp + 1040 + hb + hb * 2, sizeof ps);
            ref_post_unpack(q, &ps);
        }
    }
    free(blob);
    return e;
}

int nnsp_cascade_totals(nnsp_cascade *c, long long *chunks, long long *rounds, long long *frames_run, double *fe_ms,
                        double *chunk_ms)
{
    if (!c) return NNSP_EINVAL;
    TRY(book_take(c));
    if (chunks) *chunks = c->tot_chunks;
    if (rounds) *rounds = c->tot_rounds;
    if (frames_run) *frames_run = (long long)c->tot_frames;
    if (fe_ms) *fe_ms = c->tot_fe_ms;
    if (chunk_ms) *chunk_ms = c->tot_chunk_ms;
    return 0;
}

int nnsp_cascade_totals_reset(nnsp_cascade *c)
{
    if (!c) return NNSP_EINVAL;
    TRY(book_take(c));
    c->tot_chunks = c->tot_rounds = 0;
    c->tot_frames = 0;
    c->tot_fe_ms = c->tot_chunk_ms = 0.0;
    return 0;
}
