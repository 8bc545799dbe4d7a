/*
 * nnsp_cascade.c -- batched nnCntrlClass (include/nnsp_cascade.h).
 *
 * Per chunk: casc_begin lists every stream under the net at its position;
 * then rounds of { for each net with listed streams: one segment run of the
 * batch engine (fe -> proj -> recur -> context/tail roll) from each stream's
 * segment start to the end of the chunk; casc_control replays the
 * controller over the round's triggers, cuts each stream's segment at its
 * first net switch, requests the departing net's reset and lists the stream
 * for the next round; the resets run } until no stream is listed; finally
 * the PCM history (the voice buffer the look-back reads) rolls forward.
 * The host reads back three list lengths per round and nothing else.
 */
#include <stdlib.h>
#include <string.h>

#include "../../../include/nnsp_cascade.h"
#include "nnsp_host.h"

#define TRY(x)                 \
    do {                       \
        int _e = (x);          \
        if (_e) return _e;     \
    } while (0)

#define HIST_MAX 99   /* PcmBufClass keeps 100 frames: look-back 0..99 */

struct nnsp_cascade {
    nnsp_batch *net[3];
    int S, Tmax, H;
    int lookback[3];
    CascArgs a;                     /* persistent device pointers */
    CascState *d_st;
    int32_t *d_seg_begin, *d_counts;
    unsigned long long *d_frames;
    int16_t *d_trig[3], *d_out3[3];
    uint8_t *d_mask[3];
    int32_t *d_list[3];
    int16_t *d_hist[2];
    int hist_cur;
    int16_t *d_pcm, *d_det, *d_o3;
    int8_t *d_ran;
    void *stream;
    void *ev[2];
    int last_rounds;
    int window;                     /* frames per stream and round (0: to the chunk end) */
    float fe_ms[3], nn_ms[3];       /* last chunk, per net id: device time of fe / proj+recur */
    int runs[3];                    /* last chunk, per net id: segment runs (fe launches) */
};

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
    c->lookback[0] = p->frs_vbufBk_s2i;
    c->lookback[1] = 0; /* VAD reads the current frame (nnCntrlClass.c:243-247) */
    c->lookback[2] = p->frs_vbufBk_kws;
    c->H = c->lookback[0] > c->lookback[2] ? c->lookback[0] : c->lookback[2];
    if (c->H < 1) c->H = 1;
    const size_t S = (size_t)c->S, T = (size_t)c->Tmax;
    if ((e = nnspk_stream_create(&c->stream))) goto fail;
    for (int i = 0; i < 2; ++i)
        if ((e = nnspk_event_create(&c->ev[i]))) goto fail;
    if ((e = nnspk_malloc((void **)&c->d_st, S * sizeof(CascState)))) goto fail;
    if ((e = nnspk_malloc((void **)&c->d_seg_begin, S * 4))) goto fail;
    if ((e = nnspk_malloc((void **)&c->d_counts, 3 * 4))) goto fail;
    if ((e = nnspk_malloc((void **)&c->d_frames, 3 * 8))) goto fail;
    for (int i = 0; i < 3; ++i) {
        if ((e = nnspk_malloc((void **)&c->d_trig[i], S * T * 2))) goto fail;
        if ((e = nnspk_malloc((void **)&c->d_out3[i], S * T * 6))) goto fail;
        if ((e = nnspk_malloc((void **)&c->d_mask[i], S))) goto fail;
        if ((e = nnspk_malloc((void **)&c->d_list[i], S * 4))) goto fail;
        if ((e = nnspk_memset(c->d_mask[i], 0, S, c->stream))) goto fail;
    }
    for (int i = 0; i < 2; ++i)
        if ((e = nnspk_malloc((void **)&c->d_hist[i], S * (size_t)c->H * 320))) goto fail;
    if ((e = nnspk_memset(c->d_st, 0, S * sizeof(CascState), c->stream))) goto fail; /* pos 0 */
    {
        CascArgs *a = &c->a;
        memset(a, 0, sizeof *a);
        a->S = c->S;
        a->len_seq = len_seq;
        a->timeout_kws = p->thresh_timeout_kws;
        a->timeout_s2i = p->thresh_timeout_s2i;
        for (int i = 0; i < len_seq; ++i) a->seq[i] = seq[i];
        a->st = c->d_st;
        a->seg_begin = c->d_seg_begin;
        a->counts = c->d_counts;
        a->frames = c->d_frames;
        for (int i = 0; i < 3; ++i) {
            a->trig[i] = c->d_trig[i];
            a->out3[i] = c->d_out3[i];
            a->feats[i] = nets[i]->d_feats;
            a->prev5[i] = nets[i]->d_prev5;
            a->reset_mask[i] = c->d_mask[i];
            a->list[i] = c->d_list[i];
        }
    }
    c->window = 12;
    {
        const char *w = getenv("NNSP_CASCADE_WINDOW");
        if (w) c->window = atoi(w);
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
    void *bufs[] = {c->d_st,      c->d_seg_begin, c->d_counts,  c->d_frames,  c->d_trig[0], c->d_trig[1],
                    c->d_trig[2], c->d_out3[0],   c->d_out3[1], c->d_out3[2], c->d_mask[0], c->d_mask[1],
                    c->d_mask[2], c->d_list[0],   c->d_list[1], c->d_list[2], c->d_hist[0], c->d_hist[1],
                    c->d_pcm,     c->d_det,       c->d_o3,      c->d_ran};
    for (size_t i = 0; i < sizeof bufs / sizeof bufs[0]; ++i) nnspk_free(bufs[i]);
    for (int i = 0; i < 2; ++i) nnspk_event_destroy(c->ev[i]);
    nnspk_stream_destroy(c->stream);
    free(c);
}

int nnsp_cascade_reset(nnsp_cascade *c, const uint8_t *mask)
{
    if (!c) return NNSP_EINVAL;
    TRY(nnspk_sync(c->stream));
    for (int i = 0; i < 3; ++i) TRY(nnsp_batch_reset(c->net[i], mask)); /* synchronous */
    const uint8_t *dm = NULL;
    if (mask) {
        TRY(nnspk_h2d(c->d_mask[0], mask, (size_t)c->S, c->stream));
        dm = c->d_mask[0];
    }
    TRY(nnspk_launch_casc_reset(c->d_st, c->d_hist[c->hist_cur], c->H, dm, c->S, c->stream));
    if (mask) TRY(nnspk_memset(c->d_mask[0], 0, (size_t)c->S, c->stream));
    return nnspk_sync(c->stream);
}

int nnsp_cascade_exec_device(nnsp_cascade *c, const int16_t *pcm, int T, int8_t *net_ran, int16_t *detected,
                             int16_t *outputs3)
{
    if (!c || !pcm || T <= 0 || T > c->Tmax) {
        nnsp_set_error("nnsp_cascade_exec: T must be in 1..%d", c ? c->Tmax : 0);
        return NNSP_EINVAL;
    }
    CascArgs a = c->a;
    a.T = T;
    a.seg_len = c->window;
    a.net_ran = net_ran;
    a.detected = detected;
    a.outputs3 = outputs3;
    int32_t cnt[3];
    TRY(nnspk_event_record(c->ev[0], c->stream));
    TRY(nnspk_memset(c->d_counts, 0, 12, c->stream));
    TRY(nnspk_memset(c->d_frames, 0, 3 * 8, c->stream));
    for (int n = 0; n < 3; ++n) {
        c->fe_ms[n] = c->nn_ms[n] = 0.f;
        c->runs[n] = 0;
    }
    TRY(nnspk_launch_casc_begin(&a, c->stream));
    TRY(nnspk_d2h(cnt, c->d_counts, 12, c->stream));
    TRY(nnspk_sync(c->stream));
    int rounds = 0;
    const int16_t *hist = c->d_hist[c->hist_cur];
    while (cnt[0] + cnt[1] + cnt[2] > 0) {
        int ran[3];
        for (int n = 0; n < 3; ++n) {
            ran[n] = cnt[n] > 0;
            if (!cnt[n]) continue;
            c->runs[n]++;
            nnsp_batch *b = c->net[n];
            nnsp_segment seg;
            memset(&seg, 0, sizeof seg);
            seg.list = c->d_list[n];
            seg.n_list = cnt[n];
            seg.seg_begin = c->d_seg_begin;
            seg.lookback = c->lookback[n];
            seg.hist = hist;
            seg.hist_frames = c->H;
            seg.out3 = c->d_out3[n];
            seg.seg_len = c->window;
            TRY(nnsp_batch_run(b, pcm, T, c->d_trig[n], NULL, &seg, c->stream, 1));
        }
        TRY(nnspk_memset(c->d_counts, 0, 12, c->stream));
        TRY(nnspk_launch_casc_control(&a, c->stream));
        for (int n = 0; n < 3; ++n) {
            nnsp_batch *b = c->net[n];
            /* NNSPClass_reset of the departing streams (slot 5 already set) */
            TRY(nnspk_launch_fe_default(b->d_prev5, b->d_tail, b->d_mean, b->d_stdR, b->norm_shift,
                                        c->d_mask[n], c->S, c->stream));
            TRY(nnspk_launch_nn_default(b->d_h, b->d_c, b->d_post, b->im.img.n_lstm ? b->im.img.n_lstm : 1,
                                        c->d_mask[n], c->S, c->stream));
            TRY(nnspk_memset(c->d_mask[n], 0, (size_t)c->S, c->stream));
        }
        TRY(nnspk_d2h(cnt, c->d_counts, 12, c->stream));
        TRY(nnspk_sync(c->stream));
        for (int n = 0; n < 3; ++n) {   /* kernel times of this round's segment runs */
            if (!ran[n]) continue;
            float fe = 0.f, nn = 0.f;
            TRY(nnspk_event_elapsed(&fe, c->net[n]->ev[0], c->net[n]->ev[1]));
            TRY(nnspk_event_elapsed(&nn, c->net[n]->ev[1], c->net[n]->ev[2]));
            c->fe_ms[n] += fe;
            c->nn_ms[n] += nn;
        }
        ++rounds;
    }
    /* voice buffer: keep the last H frames for the next chunk's look-back */
    TRY(nnspk_launch_hist_roll(c->d_hist[c->hist_cur ^ 1], hist, pcm, c->S, T, c->H, c->stream));
    c->hist_cur ^= 1;
    TRY(nnspk_event_record(c->ev[1], c->stream));
    c->last_rounds = rounds;
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
    if (!c || frames < 0) return NNSP_EINVAL;
    c->window = frames;
    return 0;
}

int nnsp_cascade_sync(nnsp_cascade *c) { return c ? nnspk_sync(c->stream) : NNSP_EINVAL; }
void *nnsp_cascade_stream(nnsp_cascade *c) { return c ? c->stream : NULL; }

int nnsp_cascade_last_stats(nnsp_cascade *c, int *rounds, long long *frames_run, float *ms)
{
    if (!c) return NNSP_EINVAL;
    TRY(nnspk_sync(c->stream));
    if (rounds) *rounds = c->last_rounds;
    if (frames_run) {
        unsigned long long f[3] = {0, 0, 0};
        TRY(nnspk_d2h(f, c->d_frames, 3 * 8, c->stream));
        TRY(nnspk_sync(c->stream));
        *frames_run = (long long)(f[0] + f[1] + f[2]);
    }
    if (ms) TRY(nnspk_event_elapsed(ms, c->ev[0], c->ev[1]));
    return 0;
}

int nnsp_cascade_last_net_stats(nnsp_cascade *c, int nn_id, long long *frames_run, float *fe_ms, float *nn_ms,
                                int *launches)
{
    if (!c || nn_id < 0 || nn_id > 2) return NNSP_EINVAL;
    TRY(nnspk_sync(c->stream));
    if (frames_run) {
        unsigned long long f[3] = {0, 0, 0};
        TRY(nnspk_d2h(f, c->d_frames, 3 * 8, c->stream));
        TRY(nnspk_sync(c->stream));
        *frames_run = (long long)f[nn_id];
    }
    if (fe_ms) *fe_ms = c->fe_ms[nn_id];
    if (nn_ms) *nn_ms = c->nn_ms[nn_id];
    if (launches) *launches = c->runs[nn_id];
    return 0;
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
