/*
 * nnsp_legacy.c -- the drop-in single-stream ns-nnsp C API (nnsp_api.h) on
 * MI355X.
 *
 * Semantics follow the reference call by call (file:line cited per function);
 * the caller-owned structs (NNSPClass, FeatureClass, NeuralNetClass h/c arrays)
 * stay the source of truth: every call uploads the state it needs, runs the
 * same gfx950 kernels as the batched engine on a batch of one, and writes the
 * new state back into the structs.  Nothing is computed on the CPU; host code
 * here only moves bytes (buffer shifts, struct fields).  Like the reference
 * (global scratch, T8) this layer is not re-entrant.
 *
 * The function addresses fc_8x16 / lstm_8x16 / *_acc32b / tanh_fix /
 * sigmoid_fix / relu6_fix / linear_fix double as the layer / activation tags
 * that def_nn*.c store in NeuralNetClass and that nnsp_image.c reads.
 */
#define _POSIX_C_SOURCE 199309L /* clock_gettime (the development probe) */
#include <setjmp.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "nnsp_host.h"

/* ---------------------------------------------------------------------------
 * per-process GPU context: one HIP stream + a bump-allocated scratch arena
 * that grows on demand (a call that needs more scratch gets a larger arena;
 * the old one is freed at the start of the next call, once nothing in flight
 * uses it), and the sticky error of the last failed call
 * ------------------------------------------------------------------------- */
#define NNSP_WORKERS 4
#define DMB_IN 4096                                  /* G.dmb: mailboxes [0, 256), the inputs from 4 KiB */
#define DMB_BYTES (DMB_IN + (64u << 10))
static struct {
    void *stream;
    uint8_t *arena;
    uint8_t *retired[8]; /* arenas outgrown during the current call (their pointers may be live) */
    int n_retired;
    size_t cap, used;
    int ready;
    int depth;   /* nesting of public entry points (the outermost holds jb) */
    jmp_buf jb;
    int sticky;  /* first error since nnsp_legacy_clear(); 0 = none */
    int port;    /* 1: the reference's ARM_OPTIMIZED=0 build (row N4); 2: not yet read */
    uint8_t *hpin;  /* pinned host staging of NNSPClass_exec (NNSP_DROPIN_COPY=1: one upload, one download) */
    size_t hpin_cap;
    /* the same staging in mapped, coherent host memory: the front-end kernel
     * reads the call's inputs from it and the NN kernel writes the results to
     * it, in place of the two copies (NNSP_DROPIN_COPY=1: the copies) */
    uint8_t *hmap, *hmap_dev;
    int copy;
    /* how NNSPClass_exec waits for its launch (NNSP_DROPIN_WAIT): 2 (default)
     * polling a completion word the kernel stores after its results (the
     * mapped path only), 1 polling the stream, 0 the stream's synchronisation.
     * Median us per frame VAD / KWS / S2I: 32.4 / 34.8 / 38.7 (2), 36.6 /
     * 39.3 / 43.3 (1), 35.9 / 38.6 / 42.4 (0), profiles/r05/dropin_wait/ */
    int wait;
    /* NNSP_DROPIN_LDS (default 1): the drop-in kernel runs the call out of LDS
     * (inputs copied in there, weights staged beside them; NnRun.st_bytes) */
    int lds;
    /* NNSP_DROPIN_KARG (default 1, with NNSP_DROPIN_LDS): the inputs travel in the
     * kernel arguments (device memory) instead of being read from mapped host memory */
    int karg;
    int probe;      /* NNSP_DROPIN_PROBE=1 (PROBES builds): the drop-in kernel's phase clocks, nnsp_dropin_probes */
    /* NNSP_DROPIN_WORKER (default 1, with NNSP_DROPIN_LDS and the completion
     * word): calls go to a resident worker workgroup that keeps the net in LDS
     * (dropin_worker_kernel) instead of one launch each; it leaves after
     * NNSP_DROPIN_IDLE_MS (default 50) without a request */
    int worker;
    long long idle_ns;
    /* the workers' mailboxes and the calls' inputs in fine-grained device
     * memory the host writes (NNSP_DROPIN_DEVMBOX, default 1; NULL: in the
     * mapped staging): the worker polls and reads them without a trip across
     * PCIe (profiles/r06/devmbox/: 6.45 -> 5.35 us a round trip) */
    uint8_t *dmb;
    struct dropin_worker {
        void *stream;
        FeArgs a;   /* the arguments it serves (r.done_seq 0) */
        NnImage img;
        NnRun r;
        int live;
        long long last; /* host clock of its last request, ns */
    } W[NNSP_WORKERS];
    uint32_t seq;
    void *fetab[2]; /* the front end's prebuilt tables, per build (shipped, portable); built on first use */
} G = {.port = 2};
static void workers_stop(void);

/* The build the drop-in API reproduces: the reference selects it at compile
 * time (ARM_OPTIMIZED, ambiq_nnsp_debug.h:4); here nnsp_set_arm_optimized()
 * or, before the first call, the environment (NNSP_ARM_OPTIMIZED=0). */
static int port_on(void)
{
    if (G.port == 2) {
        const char *e = getenv("NNSP_ARM_OPTIMIZED");
        G.port = e && e[0] == '0' && e[1] == 0;
    }
    return G.port;
}

int nnsp_set_arm_optimized(int arm_optimized)
{
    if (arm_optimized != 0 && arm_optimized != 1) return NNSP_EINVAL;
    G.port = !arm_optimized;
    return 0;
}

int nnsp_get_arm_optimized(void) { return !port_on(); }

static void fail(int code, const char *what)
{
    if (!G.sticky) G.sticky = code;
    nnsp_set_error("libnnsp_mi355x (legacy API): %s failed: %s", what,
                   code > 0 ? nnspk_error_string(code) : (code == NNSP_ENOMEM ? "out of memory" : "invalid argument"));
    fprintf(stderr, "%s\n", nnsp_last_error());
    if (G.depth > 0) longjmp(G.jb, 1);
    abort(); /* unreachable: every GPU path runs inside a public entry point */
}

#define CK(x)                     \
    do {                          \
        int _e = (x);             \
        if (_e) fail(_e, #x);     \
    } while (0)

int nnsp_legacy_status(void) { return G.sticky; }

/* development probe (not in the public header): the last drop-in call's
 * phase clocks (NnRun.probe: 16 s_memrealtime values, 100 MHz) from the mapped
 * staging; 0 when NNSP_DROPIN_PROBE is off or no call ran */
int nnsp_dropin_probes(long long *out)
{
    if (!G.ready || !G.probe || G.copy || !out) return NNSP_EINVAL;
    memcpy(out, G.hmap + G.hpin_cap - 16 - NNSP_PROBE_BYTES, NNSP_PROBE_BYTES);
    return 0;
}
void nnsp_legacy_clear(void) { G.sticky = 0; }

static int gctx(void)
{
    if (G.ready) return 0;
    int e = nnspk_stream_create(&G.stream);
    if (e) return e;
    G.cap = 4u << 20;
    if ((e = nnspk_malloc((void **)&G.arena, G.cap))) return e;
    G.hpin_cap = 64u << 10;
    if ((e = nnspk_host_alloc((void **)&G.hpin, G.hpin_cap))) return e;
    {
        const char *cp = getenv("NNSP_DROPIN_COPY");
        G.copy = cp && atoi(cp) != 0;
        const char *wt = getenv("NNSP_DROPIN_WAIT");
        G.wait = wt ? atoi(wt) : 2;
        const char *pb = getenv("NNSP_DROPIN_PROBE");
        G.probe = pb && atoi(pb) != 0;
        const char *ld = getenv("NNSP_DROPIN_LDS");
        G.lds = !ld || atoi(ld) != 0;
        const char *ka = getenv("NNSP_DROPIN_KARG");
        G.karg = !ka || atoi(ka) != 0;
        const char *wk = getenv("NNSP_DROPIN_WORKER");
        G.worker = !wk || atoi(wk) != 0;
        const char *dm = getenv("NNSP_DROPIN_DEVMBOX");
        if (!dm || atoi(dm) != 0) {
            void *p = NULL;
            if (!nnspk_malloc_finegrained(&p, DMB_BYTES)) G.dmb = (uint8_t *)p;
        }
        const char *im = getenv("NNSP_DROPIN_IDLE_MS");
        const int ms = im ? atoi(im) : 50;
        G.idle_ns = (long long)(ms > 2 ? ms : 2) * 1000000LL;
    }
    if (!G.copy && (e = nnspk_host_alloc_mapped((void **)&G.hmap, (void **)&G.hmap_dev, G.hpin_cap))) return e;
    G.ready = 1;
    return 0;
}

static void *dscratch(size_t n)
{
    n = (n + 255) & ~(size_t)255;
    if (G.used + n > G.cap) {
        /* grow: pointers handed out earlier in this call stay valid -- every
         * outgrown arena of the call is retired, and all of them are freed by
         * the next begin(), after the call's synchronisation */
        if (G.n_retired == (int)(sizeof G.retired / sizeof G.retired[0]))
            fail(NNSP_ENOMEM, "legacy scratch: too many arena growths in one call");
        size_t cap = G.cap * 2;
        while (cap < n) cap *= 2;
        uint8_t *a = NULL;
        CK(nnspk_malloc((void **)&a, cap));
        G.retired[G.n_retired++] = G.arena;
        G.arena = a;
        G.cap = cap;
        G.used = 0;
    }
    void *p = G.arena + G.used;
    G.used += n;
    return p;
}

const char *nnsp_strerror(int code);

static void begin(void)
{
    CK(gctx());
    /* the previous call synchronised (fin) or failed after a sync-free
     * launch error: wait for the stream, then nothing uses the old arenas */
    if (G.n_retired) {
        workers_stop();
        nnspk_sync(G.stream);
        for (int i = 0; i < G.n_retired; ++i) nnspk_free(G.retired[i]);
        G.n_retired = 0;
    }
    G.used = 0;
}
static void *up(const void *h, size_t n)
{
    void *d = dscratch(n);
    if (h) CK(nnspk_h2d(d, h, n, G.stream));
    else CK(nnspk_memset(d, 0, n, G.stream));
    return d;
}
static void down(void *h, const void *d, size_t n) { CK(nnspk_d2h(h, d, n, G.stream)); }
static void fin(void) { CK(nnspk_sync(G.stream)); }

/* NNSP_DROPIN_WAIT=2: spin until the kernel's completion word holds seq; the
 * stream is queried now and then, so that a failed launch is reported (and a
 * completed stream without the word is an error) instead of spinning for ever */
static int wait_word_on(volatile uint32_t *w, uint32_t seq, void *stream)
{
    for (unsigned i = 1;; ++i) {
        if (*w == seq) break;
        if ((i & 255) == 0) {
            const int d = nnspk_stream_done(stream);
            if (d < 0) CK(-d);
            if (d > 0 && *w != seq) return 1;
        }
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    return 0;
}
static void wait_word(volatile uint32_t *w, uint32_t seq)
{
    if (wait_word_on(w, seq, G.stream)) fail(NNSP_EINVAL, "NNSPClass_exec: the completion word");
}

/* ---------------------------------------------------------------------------
 * device image cache.  An image is keyed by the tables' addresses, the layer
 * description and a 64-bit FNV-1a hash of the weight, recurrent-weight and
 * bias BYTES, so tables changed in place or rebuilt at reused addresses get a
 * new image (the reference reads its tables on every call).  Most recently
 * used first; at most IMG_MAX images, the least recently used freed.
 * ------------------------------------------------------------------------- */
#define IMG_MAX 32
typedef struct img_node {
    struct img_node *next;
    const void *key[4];
    int ikey[8];
    uint64_t bytes;
    nnsp_image im;
    int out_linear;
    uint8_t *blob;      /* net images: a host copy of every table byte the image was built from */
    size_t blob_n;
} img_node;
static img_node *g_imgs;

static uint64_t fnv(uint64_t h, const void *p, size_t n)
{
    const uint8_t *b = (const uint8_t *)p;
    for (size_t i = 0; i < n; ++i) {
        h ^= b[i];
        h *= 1099511628211ULL;
    }
    return h;
}

static uint64_t layer_bytes_hash(uint64_t h, const nnsp_layer_desc *d)
{
    const size_t rows = (size_t)(d->type == NN_LSTM ? 4 * d->N : d->N);
    if (d->W) h = fnv(h, d->W, rows * (size_t)d->K);
    if (d->Wr) h = fnv(h, d->Wr, rows * (size_t)d->N);
    if (d->B) h = fnv(h, d->B, rows * 2);
    return h;
}

static img_node *img_find(const void *k0, const void *k1, const void *k2, const void *k3, const int *ik,
                          uint64_t bytes)
{
    img_node *prev = NULL;
    for (img_node *n = g_imgs; n; prev = n, n = n->next)
        if (n->key[0] == k0 && n->key[1] == k1 && n->key[2] == k2 && n->key[3] == k3 &&
            !memcmp(n->ikey, ik, sizeof n->ikey) && n->bytes == bytes) {
            if (prev) { /* move to the front */
                prev->next = n->next;
                n->next = g_imgs;
                g_imgs = n;
            }
            return n;
        }
    return NULL;
}

/* blob (may be NULL): the tables' host copy, owned by the new entry -- freed
 * here when the entry cannot be built */
static img_node *img_add(const void *k0, const void *k1, const void *k2, const void *k3, const int *ik,
                         uint64_t bytes, const nnsp_layer_desc *L, int nl, int out_linear, uint8_t *blob,
                         size_t blob_n)
{
    int count = 0;
    img_node *last = NULL, *before_last = NULL;
    for (img_node *n = g_imgs; n; n = n->next) {
        ++count;
        before_last = last;
        last = n;
    }
    if (count >= IMG_MAX && last) { /* evict the least recently used (nothing in flight uses it) */
        workers_stop();
        const int se = nnspk_sync(G.stream);
        if (se) {
            free(blob);
            fail(se, "nnspk_sync");
        }
        if (before_last) before_last->next = NULL;
        else g_imgs = NULL;
        nnsp_image_free(&last->im);
        free(last->blob);
        free(last);
    }
    img_node *n = (img_node *)calloc(1, sizeof *n);
    if (!n) {
        free(blob);
        fail(NNSP_ENOMEM, "image cache entry");
    }
    n->key[0] = k0; n->key[1] = k1; n->key[2] = k2; n->key[3] = k3;
    memcpy(n->ikey, ik, sizeof n->ikey);
    n->bytes = bytes;
    int e = nnsp_image_build(&n->im, L, nl, 0, 0, 0, 1);
    if (!e) e = nnsp_image_upload(&n->im, G.stream);
    if (e) {
        nnsp_image_free(&n->im);
        free(n);
        free(blob);
        fail(e, "nnsp_image_build/upload");
    }
    n->out_linear = out_linear;
    n->blob = blob;
    n->blob_n = blob_n;
    n->next = g_imgs;
    g_imgs = n;
    return n;
}

/* the table bytes of a layer list, in order (W, Wr, B per layer): their
 * total size, and a copy into dst / a comparison with src */
static size_t layer_span(const nnsp_layer_desc *d, int which)
{
    const size_t rows = (size_t)(d->type == NN_LSTM ? 4 * d->N : d->N);
    if (which == 0) return d->W ? rows * (size_t)d->K : 0;
    if (which == 1) return d->Wr ? rows * (size_t)d->N : 0;
    return d->B ? rows * 2 : 0;
}
static const void *layer_ptr(const nnsp_layer_desc *d, int which)
{
    return which == 0 ? (const void *)d->W : (which == 1 ? (const void *)d->Wr : (const void *)d->B);
}
static size_t tables_bytes(const nnsp_layer_desc *L, int nl)
{
    size_t n = 0;
    for (int i = 0; i < nl; ++i)
        for (int w = 0; w < 3; ++w) n += layer_span(&L[i], w);
    return n;
}
static int tables_equal(const uint8_t *blob, size_t blob_n, const nnsp_layer_desc *L, int nl)
{
    size_t o = 0;
    for (int i = 0; i < nl; ++i)
        for (int w = 0; w < 3; ++w) {
            const size_t n = layer_span(&L[i], w);
            if (!n) continue;
            if (o + n > blob_n || memcmp(blob + o, layer_ptr(&L[i], w), n)) return 0;
            o += n;
        }
    return o == blob_n;
}
static void tables_copy(uint8_t *blob, const nnsp_layer_desc *L, int nl)
{
    for (int i = 0; i < nl; ++i)
        for (int w = 0; w < 3; ++w) {
            const size_t n = layer_span(&L[i], w);
            if (n) memcpy(blob, layer_ptr(&L[i], w), n);
            blob += n;
        }
}

/* A NeuralNetClass's device image: keyed by its address and a hash of its
 * shape, qbits, layer / activation functions and table pointers; the tables'
 * bytes are compared with the copy the image was built from (memcmp: the
 * reference reads its tables on every call, so tables rewritten in place get
 * a new image -- a byte-wise hash of them was ~30 % of a drop-in S2I frame) */
/* check 0: a cached image without the comparison of the tables' bytes (*fresh
 * 0; NNSPClass_exec compares them while the call runs, net_tables_match), 1 when
 * built here */
static img_node *net_image_ex(const NeuralNetClass *net, int check, int *fresh)
{
    if (fresh) *fresh = 0;
    uint64_t h = 1469598103934665603ULL;
#define MIX(v)                                   \
    do {                                         \
        h ^= (uint64_t)(uintptr_t)(v);           \
        h *= 1099511628211ULL;                   \
    } while (0)
    MIX(net->numlayers);
    MIX(port_on());
    for (int i = 0; i < net->numlayers && i < NN_MAX_LAYERS; ++i) {
        MIX(net->size_layer[i]); MIX(net->size_layer[i + 1]); MIX(net->net_layer_type[i]);
        MIX(net->qbit_kernel[i]); MIX(net->qbit_input[i]); MIX(net->qbit_bias[i]); MIX(net->activation_type[i]);
        MIX(net->act_func[i]); MIX(net->layer_func[i]); MIX(net->pt_kernel[i]); MIX(net->pt_bias[i]);
        MIX(net->pt_kernel_rec[i]);
    }
#undef MIX
    nnsp_layer_desc L[NN_MAX_LAYERS];
    int nl = 0, lin = 0;
    CK(nnsp_describe_net(net, L, &nl, &lin));
    for (int i = 0; i < nl; ++i) L[i].portable = port_on();
    const int ik[8] = {(int)(h & 0xffffffffu), (int)(h >> 32), net->numlayers, 0, 0, 0, 0, 0};
    img_node *n = img_find(net, NULL, NULL, NULL, ik, 0);
    if (n && (!check || tables_equal(n->blob, n->blob_n, L, nl))) return n;
    if (n) { /* tables changed in place: this image is stale */
        workers_stop();
        CK(nnspk_sync(G.stream));
        g_imgs = n->next; /* img_find moved it to the front */
        nnsp_image_free(&n->im);
        free(n->blob);
        free(n);
    }
    const size_t nb = tables_bytes(L, nl);
    uint8_t *blob = (uint8_t *)malloc(nb ? nb : 1);
    if (!blob) fail(NNSP_ENOMEM, "image cache tables copy");
    tables_copy(blob, L, nl);
    if (fresh) *fresh = 1;
    return img_add(net, NULL, NULL, NULL, ik, 0, L, nl, lin, blob, nb);
}
static img_node *net_image(const NeuralNetClass *net) { return net_image_ex(net, 1, NULL); }
/* the net's tables still hold the bytes image n was built from */
static int net_tables_match(const NeuralNetClass *net, const img_node *n)
{
    nnsp_layer_desc L[NN_MAX_LAYERS];
    int nl = 0, lin = 0;
    CK(nnsp_describe_net(net, L, &nl, &lin));
    return tables_equal(n->blob, n->blob_n, L, nl);
}

/* LSTM h/c of a NeuralNetClass <-> device rows [l][hs] (hs: the widest
 * LSTM rounded up to 8; NnRun.hs) */
static int net_hs(const NeuralNetClass *net)
{
    int hs = 8;
    for (int i = 0; i < net->numlayers && i < NN_MAX_LAYERS; ++i)
        if (net->net_layer_type[i] == lstm && net->size_layer[i + 1] > hs) hs = (net->size_layer[i + 1] + 7) / 8 * 8;
    return hs;
}

static void net_state_up(const NeuralNetClass *net, int hs, int16_t **dh, int32_t **dc)
{
    static int16_t h[NN_MAX_LSTM * (NN_MAX_WIDTH + 8)];
    static int32_t c[NN_MAX_LSTM * (NN_MAX_WIDTH + 8)];
    memset(h, 0, sizeof h);
    memset(c, 0, sizeof c);
    int l = 0;
    for (int i = 0; i < net->numlayers && l < NN_MAX_LSTM; ++i)
        if (net->net_layer_type[i] == lstm) {
            const int N = net->size_layer[i + 1];
            memcpy(h + (size_t)l * hs, net->pt_hstate[i], (size_t)N * 2);
            memcpy(c + (size_t)l * hs, net->pt_cstate[i], (size_t)N * 4);
            ++l;
        }
    *dh = (int16_t *)up(h, (size_t)(l ? l : 1) * hs * 2);
    *dc = (int32_t *)up(c, (size_t)(l ? l : 1) * hs * 4);
}

static void net_state_down(NeuralNetClass *net, int hs, const int16_t *dh, const int32_t *dc)
{
    static int16_t h[NN_MAX_LSTM * (NN_MAX_WIDTH + 8)];
    static int32_t c[NN_MAX_LSTM * (NN_MAX_WIDTH + 8)];
    int nls = 0;
    for (int i = 0; i < net->numlayers && i < NN_MAX_LAYERS; ++i) nls += net->net_layer_type[i] == lstm;
    if (nls > NN_MAX_LSTM) nls = NN_MAX_LSTM;
    if (nls) {
        down(h, dh, (size_t)nls * hs * 2);
        down(c, dc, (size_t)nls * hs * 4);
    }
    fin();
    int l = 0;
    for (int i = 0; i < net->numlayers && l < NN_MAX_LSTM; ++i)
        if (net->net_layer_type[i] == lstm) {
            const int N = net->size_layer[i + 1];
            memcpy(net->pt_hstate[i], h + (size_t)l * hs, (size_t)N * 2);
            memcpy(net->pt_cstate[i], c + (size_t)l * hs, (size_t)N * 4);
            ++l;
        }
}

/* ---------------------------------------------------------------------------
 * activations (activation.c)
 * ------------------------------------------------------------------------- */
static void *act_call(int type, int32_t *x, void *y, int len)
{
    if (len <= 0) return y;
    begin();
    const size_t ob = (size_t)len * (type == 3 ? 4 : 2);
    int32_t *dx = (int32_t *)up(x, (size_t)len * 4);
    void *dy = up(NULL, ob);
    CK(nnspk_launch_act(type, dx, dy, len, G.stream));
    down(y, dy, ob);
    fin();
    return (char *)y + ob;
}
static void *relu6_fix_impl(int16_t *y, int32_t *x, int len) { return act_call(0, x, y, len); }
static void *tanh_fix_impl(int16_t *y, int32_t *x, int len) { return act_call(1, x, y, len); }
static void *sigmoid_fix_impl(int16_t *y, int32_t *x, int len) { return act_call(2, x, y, len); }
static void *linear_fix_impl(int32_t *y, int32_t *x, int len) { return act_call(3, x, y, len); }

/* ---------------------------------------------------------------------------
 * layers (affine.c:409-490, lstm.c:15-214) -- single-layer images
 * ------------------------------------------------------------------------- */
static int run_layer(int type, int acc32, int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec,
                     int16_t *p_bias, int16_t *input, int16_t *h_state, int32_t *c_state,
                     int16_t dim_output, int16_t dim_input, int16_t qk, int16_t qb, int16_t qi,
                     int16_t qir, void *(*act)(void *, int32_t *, int))
{
    begin();
    nnsp_layer_desc d;
    memset(&d, 0, sizeof d);
    d.type = type;
    d.K = dim_input;
    d.N = dim_output;
    d.acc32 = acc32;
    d.qk = qk; d.qb = qb; d.qi = qi; d.qir = qir;
    d.W = p_kernel; d.Wr = p_kernel_rec; d.B = p_bias;
    d.portable = port_on();
    d.act = type == NN_LSTM ? 1 : nnsp_act_of(act);
    if (d.act < 0) {
        fprintf(stderr, "libnnsp_mi355x: unsupported activation function pointer\n");
        return -1;
    }
    const int ik[8] = {type, acc32, dim_output, dim_input, qk, qb, qi, (qir << 4) | d.act};
    const uint64_t bytes = layer_bytes_hash(1469598103934665603ULL, &d) ^ (d.portable ? 0x9e3779b97f4a7c15ULL : 0);
    img_node *n = img_find(p_kernel, p_kernel_rec, p_bias, (void *)(intptr_t)0x1a7e, ik, bytes);
    if (!n) n = img_add(p_kernel, p_kernel_rec, p_bias, (void *)(intptr_t)0x1a7e, ik, bytes, &d, 1, d.act == 3, NULL, 0);
    int16_t in_pad[NN_MAX_K];
    memset(in_pad, 0, sizeof in_pad);
    memcpy(in_pad, input, (size_t)dim_input * 2);
    int16_t *din = (int16_t *)up(in_pad, sizeof in_pad);
    int16_t hs[NN_MAX_K];
    int32_t cs[NN_MAX_K];
    memset(hs, 0, sizeof hs);
    memset(cs, 0, sizeof cs);
    if (type == NN_LSTM) {
        memcpy(hs, h_state, (size_t)dim_output * 2);
        memcpy(cs, c_state, (size_t)dim_output * 4);
    }
    int16_t *dh = (int16_t *)up(hs, sizeof hs);
    int32_t *dc = (int32_t *)up(cs, sizeof cs);
    int32_t *dout = (int32_t *)up(NULL, NN_MAX_K * 4);
    NnRun r;
    memset(&r, 0, sizeof r);
    r.S = 1; r.T = 1; r.mode = NN_MODE_DIRECT; r.nl_run = 1;
    r.direct_in = din; r.h = dh; r.c = dc; r.logits = dout; r.out_stride = NN_MAX_K;
    r.hs = NN_MAX_K;
    CK(nnspk_launch_nn(&n->im.img, &r, G.stream));
    down(p_output, dout, (size_t)dim_output * (n->out_linear ? 4 : 2));
    if (type == NN_LSTM) {
        down(hs, dh, sizeof hs);
        down(cs, dc, sizeof cs);
    }
    fin();
    if (type == NN_LSTM) {
        memcpy(h_state, hs, (size_t)dim_output * 2);
        memcpy(c_state, cs, (size_t)dim_output * 4);
    }
    return 0;
}

static int fc_8x16_impl(int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias,
            int16_t *input, int16_t *input_rec, int32_t *c_state, int16_t dim_output,
            int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel, int16_t qbit_bias,
            int16_t qbit_input, int16_t qbit_input_rec, ACTIVATION_TYPE act_type,
            void *(*act)(void *, int32_t *, int))
{
    (void)input_rec; (void)c_state; (void)dim_input_rec; (void)act_type;
    return run_layer(NN_FC, 0, p_output, p_kernel, p_kernel_rec, p_bias, input, NULL, NULL,
                     dim_output, dim_input, qbit_kernel, qbit_bias, qbit_input, qbit_input_rec, act);
}

static int fc_8x16_acc32b_impl(int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias,
                   int16_t *input, int16_t *input_rec, int32_t *c_state, int16_t dim_output,
                   int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel,
                   int16_t qbit_bias, int16_t qbit_input, int16_t qbit_input_rec,
                   ACTIVATION_TYPE act_type, void *(*act)(void *, int32_t *, int))
{
    (void)input_rec; (void)c_state; (void)dim_input_rec; (void)act_type;
    return run_layer(NN_FC, 1, p_output, p_kernel, p_kernel_rec, p_bias, input, NULL, NULL,
                     dim_output, dim_input, qbit_kernel, qbit_bias, qbit_input, qbit_input_rec, act);
}

static int lstm_8x16_impl(int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias,
              int16_t *input, int16_t *h_state, int32_t *c_state, int16_t dim_output,
              int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel, int16_t qbit_bias,
              int16_t qbit_input, int16_t qbit_input_rec, ACTIVATION_TYPE act_type,
              void *(*act)(void *, int32_t *, int))
{
    (void)dim_input_rec; (void)act_type; (void)act;
    return run_layer(NN_LSTM, 0, p_output, p_kernel, p_kernel_rec, p_bias, input, h_state, c_state,
                     dim_output, dim_input, qbit_kernel, qbit_bias, qbit_input, qbit_input_rec, NULL);
}

static int lstm_8x16_acc32b_impl(int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias,
                     int16_t *input, int16_t *h_state, int32_t *c_state, int16_t dim_output,
                     int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel,
                     int16_t qbit_bias, int16_t qbit_input, int16_t qbit_input_rec,
                     ACTIVATION_TYPE act_type, void *(*act)(void *, int32_t *, int))
{
    (void)dim_input_rec; (void)act_type; (void)act;
    return run_layer(NN_LSTM, 1, p_output, p_kernel, p_kernel_rec, p_bias, input, h_state, c_state,
                     dim_output, dim_input, qbit_kernel, qbit_bias, qbit_input, qbit_input_rec, NULL);
}

/* ---------------------------------------------------------------------------
 * NeuralNetClass (neural_nets.c:22-168)
 * ------------------------------------------------------------------------- */
void NeuralNetClass_init(NeuralNetClass *pt_inst) { (void)pt_inst; }

void NeuralNetClass_setDefault(NeuralNetClass *pt_inst)
{
    for (int i = 0; i < pt_inst->numlayers; ++i)
        if (pt_inst->net_layer_type[i] == lstm) {
            memset(pt_inst->pt_cstate[i], 0, (size_t)pt_inst->size_layer[i + 1] * 4);
            memset(pt_inst->pt_hstate[i], 0, (size_t)pt_inst->size_layer[i + 1] * 2);
        }
}

static void NeuralNetClass_exe_impl(NeuralNetClass *pt_inst, int16_t *input, int32_t *output, int8_t debug_layer)
{
    const int nl = debug_layer < 0 ? pt_inst->numlayers : debug_layer;
    if (nl == 0) { /* neural_nets.c:85-91: copy the input through */
        memcpy(output, input, (size_t)pt_inst->size_layer[0] * 2);
        return;
    }
    begin();
    img_node *n = net_image(pt_inst);
    int16_t in_pad[NN_MAX_K];
    memset(in_pad, 0, sizeof in_pad);
    memcpy(in_pad, input, (size_t)pt_inst->size_layer[0] * 2);
    int16_t *din = (int16_t *)up(in_pad, sizeof in_pad);
    int16_t *dh;
    int32_t *dc;
    const int hs = net_hs(pt_inst);
    net_state_up(pt_inst, hs, &dh, &dc);
    int32_t *dout = (int32_t *)up(NULL, NN_MAX_K * 4);
    NnRun r;
    memset(&r, 0, sizeof r);
    r.S = 1; r.T = 1; r.mode = NN_MODE_DIRECT; r.nl_run = nl;
    r.direct_in = din; r.h = dh; r.c = dc; r.logits = dout; r.out_stride = NN_MAX_K;
    r.hs = hs;
    CK(nnspk_launch_nn(&n->im.img, &r, G.stream));
    const int lin = pt_inst->activation_type[nl - 1] == linear;
    down(output, dout, (size_t)pt_inst->size_layer[nl] * (lin ? 4 : 2));
    net_state_down(pt_inst, hs, dh, dc);
}

/* ---------------------------------------------------------------------------
 * front end (spectrogram_module.c, feature_module.c, melSpecProc.c, fixlog10.c,
 * fft_arm.c)
 * ------------------------------------------------------------------------- */
int stftModule_construct(stftModule *ps) /* spectrogram_module.c:14-24 */
{
    ps->len_win = len_stft_win_coeff;
    ps->hop = hop;
    ps->len_fft = LEN_FFT_NNSP;
    ps->window = stft_win_coeff;
    arm_fft_init();
    return 0;
}

int stftModule_setDefault(stftModule *ps) /* :25-31 */
{
    memset(ps->dataBuffer, 0, (size_t)ps->len_win * 2);
    return 0;
}

void arm_fft_init(void) { /* twiddles are compile-time tables; nothing to build */ }

static void arm_fft_exec_impl(int32_t *y, int32_t *x) /* fft_arm.c:16-20 -> arm_rfft_q31 */
{
    begin();
    int32_t *dx = (int32_t *)up(x, 512 * 4);
    int32_t *dy = (int32_t *)up(NULL, 1024 * 4);
    CK(nnspk_launch_rfft(dx, dy, 1, G.stream));
    down(y, dy, 1024 * 4);
    down(x, dx, 512 * 4); /* CMSIS transforms pSrc in place */
    fin();
}

/* one FE frame on the GPU: tail = dataBuffer[160..479] before the shift */
static void fe_frame(const int16_t *tail, const int16_t *pcm, const int32_t *mean, const int32_t *stdR,
                     int qbit, int16_t *feat40, int32_t *log40, int32_t *spec1024, int port)
{
    begin();
    FeArgs a;
    memset(&a, 0, sizeof a);
    a.port = port;
    a.pcm = (const int16_t *)up(pcm, 160 * 2);
    a.tail = (const int16_t *)up(tail, 320 * 2);
    a.S = 1; a.T = 1;
    int32_t zeros[40] = {0};
    a.mean = (const int32_t *)up(mean ? mean : zeros, 160);
    a.stdR = (const int32_t *)up(stdR ? stdR : zeros, 160);
    a.norm_shift = 30 - qbit;
    a.feats = (int16_t *)up(NULL, 80);
    if (log40) a.dbg_log = (int32_t *)up(NULL, 160);
    if (spec1024) a.dbg_spec = (int32_t *)up(NULL, 4096);
    CK(nnspk_launch_fe(&a, G.stream));
    if (feat40) down(feat40, a.feats, 80);
    if (log40) down(log40, a.dbg_log, 160);
    if (spec1024) down(spec1024, a.dbg_spec, 4096);
    fin();
}

static int stftModule_analyze_arm_impl(void *ps_, int16_t *x, int32_t *y) /* :94-124 */
{
    stftModule *ps = (stftModule *)ps_;
    int16_t tail[320];
    memcpy(tail, ps->dataBuffer + 160, sizeof tail);
    fe_frame(tail, x, NULL, NULL, 8, NULL, NULL, y, 0);
    memmove(ps->dataBuffer, ps->dataBuffer + 160, 320 * 2);
    memcpy(ps->dataBuffer + 320, x, 160 * 2);
    return 0;
}

static void spec2pspec_arm_impl(int32_t *y, int32_t *x, int len) /* :79-92 */
{
    if (len <= 0) return;
    begin();
    int32_t *dx = (int32_t *)up(x, (size_t)2 * len * 4);
    int32_t *dy = (int32_t *)up(NULL, (size_t)len * 4);   /* one vector: any len */
    CK(nnspk_launch_pspec(dy, dx, len, 1, 27, G.stream));
    down(y, dy, (size_t)len * 4);
    fin();
}

/* ---- the ARM_OPTIMIZED=0 build's front-end stages (row N4) ---- */
static int stftModule_analyze_impl(stftModule *ps, int16_t *x, int32_t *y) /* spectrogram_module.c:47-77 */
{
    int16_t tail[320];
    int32_t spec[1024];
    memcpy(tail, ps->dataBuffer + 160, sizeof tail);
    fe_frame(tail, x, NULL, NULL, 8, NULL, NULL, spec, 1);
    memcpy(y, spec, 514 * 4); /* rfft writes bins 0..256 (fft.c:27-126) */
    memmove(ps->dataBuffer, ps->dataBuffer + 160, 320 * 2);
    memcpy(ps->dataBuffer + 320, x, 160 * 2);
    return 0;
}

static void spec2pspec_impl(int32_t *y, int32_t *x, int len) /* spectrogram_module.c:33-45 */
{
    if (len <= 0) return;
    begin();
    int32_t *dx = (int32_t *)up(x, (size_t)2 * len * 4);
    int32_t *dy = (int32_t *)up(NULL, (size_t)len * 4);   /* one vector: any len */
    CK(nnspk_launch_pspec(dy, dx, len, 1, 15, G.stream));
    down(y, dy, (size_t)len * 4);
    fin();
}

static void rfft_impl(int num_rfft, int32_t *input, void *output) /* fft.c:27-126 */
{
    /* the reference's twiddle and bit-reversal tables serve 256 and 512
     * points; for other sizes it reads past them (rfft: R = 256, fft: 2^0) */
    if (num_rfft != 512 && num_rfft != 256)
        fail(NNSP_EUNSUPPORTED, "rfft: num_rfft must be 256 or 512 (the sizes fft.c's tables serve)");
    const int e = num_rfft == 512 ? 8 : 7;
    begin();
    int32_t *dx = (int32_t *)up(input, (size_t)num_rfft * 4);
    int32_t *dy = (int32_t *)up(NULL, (size_t)(num_rfft + 2) * 4);
    CK(nnspk_launch_fft_dif(dx, dy, e, 1, G.stream));
    down(output, dy, (size_t)(num_rfft + 2) * 4);
    fin();
}

static void fft_impl(int exp_nfft, void *input, void *output) /* fft.c:128-221 */
{
    if (exp_nfft < 0 || exp_nfft > 8)
        fail(NNSP_EUNSUPPORTED, "fft: exp_nfft must be 0..8 (the sizes fft.c's tables serve)");
    const size_t bytes = (size_t)8 << exp_nfft;
    begin();
    int32_t *dx = (int32_t *)up(input, bytes);
    int32_t *dy = (int32_t *)up(NULL, bytes);
    CK(nnspk_launch_fft_dif(dx, dy, exp_nfft, 0, G.stream));
    down(output, dy, bytes);
    down(input, dx, bytes); /* fft() works in place on its input (fft.c:180-195) */
    fin();
}

/* ---- complex.c (the drop-in complex.h): one k_cplx launch per call ---- */
static void cplx(int op, int32_t *out, size_t out_n, const void *a, size_t a_n, int32_t *b, size_t b_n, int shift,
                 int len, int b_back)
{
    begin();
    int32_t *da = (int32_t *)up(a, a_n * 4);
    int32_t *db = b_n ? (int32_t *)up(b, b_n * 4) : NULL;
    int32_t *dout = (int32_t *)up(NULL, out_n * 4);
    CK(nnspk_launch_cplx(op, dout, da, db, shift, len, G.stream));
    if (b_back) down(b, db, b_n * 4);
    down(out, dout, out_n * 4);
    fin();
}
static size_t nz(int len) { return len > 0 ? (size_t)len : 0; }
static void complex32_copy_impl(COMPLEX32 *dst, COMPLEX32 *src)
{
    cplx(NNSP_CPLX_COPY, &dst->real, 2, src, 2, NULL, 0, 0, 1, 0);
}
static int overlaps(const void *a, size_t an, const void *b, size_t bn)
{
    const char *pa = (const char *)a, *pb = (const char *)b;
    return pa < pb + bn && pb < pa + an;
}
static void complex32_interprod_impl(COMPLEX32 *out, COMPLEX32 *arry1, COMPLEX32 *arry2, int shift_r, int len);
static void complex32_affine_impl(COMPLEX32 *out, COMPLEX32 *Mat, COMPLEX32 *input, int shift_r, int len)
{
    if (len <= 0) return;
    /* complex.c:14-31 writes out + i row by row: when out aliases input or
     * Mat, later rows read the rows already written -- run them in that order
     * (one interprod launch per row, each on the host's updated values) */
    const size_t vb = nz(len) * sizeof(COMPLEX32);
    if (overlaps(out, vb, input, vb) || overlaps(out, vb, Mat, vb * nz(len))) {
        for (int i = 0; i < len; ++i) complex32_interprod_impl(out + i, input, Mat + (size_t)i * nz(len), shift_r, len);
        return;
    }
    cplx(NNSP_CPLX_AFFINE, &out->real, 2 * nz(len), Mat, 2 * nz(len) * nz(len), &input->real, 2 * nz(len), shift_r,
         len, 0);
}
static void complex32_interprod_impl(COMPLEX32 *out, COMPLEX32 *arry1, COMPLEX32 *arry2, int shift_r, int len)
{
    cplx(NNSP_CPLX_INTERPROD, &out->real, 2, arry2, 2 * nz(len), &arry1->real, 2 * nz(len), shift_r, len, 0);
}
static void complex32_complex16_elmtprod_impl(COMPLEX32 *out, COMPLEX32 *arry1, COMPLEX16 *arry2, int len)
{
    if (len <= 0) return;
    cplx(NNSP_CPLX_ELMTPROD, &out->real, 2 * nz(len), arry1, 2 * nz(len), (int32_t *)arry2, nz(len), 0, len, 0);
}
static void complex32_add_impl(COMPLEX32 *out, COMPLEX32 *addr1, COMPLEX32 *addr2)
{
    cplx(NNSP_CPLX_ADD, &out->real, 2, addr1, 2, &addr2->real, 2, 0, 1, 0);
}
static void complexArry32_add_impl(COMPLEX32 *out, COMPLEX32 *addr1, COMPLEX32 *addr2, int len)
{
    if (len <= 0) return;
    cplx(NNSP_CPLX_ARRY_ADD, &out->real, 2 * nz(len), addr1, 2 * nz(len), &addr2->real, 2 * nz(len), 0, len, 0);
}
static void complex32_neg_impl(COMPLEX32 *out, COMPLEX32 *in)
{
    cplx(NNSP_CPLX_NEG, &out->real, 2, in, 2, NULL, 0, 0, 1, 0);
}
static void complex32_sub_impl(COMPLEX32 *out, COMPLEX32 *a, COMPLEX32 *b)
{
    cplx(NNSP_CPLX_SUB, &out->real, 2, a, 2, &b->real, 2, 0, 1, 1);
}
static void complex32_mul_impl(COMPLEX32 *out, COMPLEX32 *addr1, COMPLEX32 *addr2)
{
    cplx(NNSP_CPLX_MUL, &out->real, 2, addr1, 2, &addr2->real, 2, 0, 1, 0);
}
static void complex32_init_impl(COMPLEX32 *inst, int32_t real, int32_t imag)
{
    const int32_t v[2] = {real, imag};
    cplx(NNSP_CPLX_INIT, &inst->real, 2, v, 2, NULL, 0, 0, 1, 0);
}
static void complex32_real2cmplx_impl(COMPLEX32 *inst, int32_t real) { complex32_init_impl(inst, real, 0); }
static void complexArry32_real2cmplx_impl(COMPLEX32 *inst, int32_t *real, int32_t len)
{
    if (len <= 0) return;
    cplx(NNSP_CPLX_ARRY_INIT, &inst->real, 2 * nz(len), real, nz(len), NULL, 0, 0, len, 0);
}
static void complexArry32_init_impl(COMPLEX32 *inst, int32_t *real, int32_t *imag, int len)
{
    if (len <= 0) return;
    cplx(NNSP_CPLX_ARRY_INIT, &inst->real, 2 * nz(len), real, nz(len), imag, nz(len), 0, len, 0);
}

static void melSpecProc_impl(int32_t *specs, int32_t *melSpecs) /* melSpecProc.c:6-27 */
{
    begin();
    int32_t *ds = (int32_t *)up(specs, 257 * 4);
    int32_t *dm = (int32_t *)up(NULL, 160);
    CK(nnspk_launch_mel(ds, dm, 1, G.stream));
    down(melSpecs, dm, 160);
    fin();
}

static void norm_oneTwo_impl(int32_t x, int32_t *y, int8_t *shift) /* fixlog10.c:9-28 */
{
    begin();
    int32_t *dx = (int32_t *)up(&x, 4);
    int32_t *dy = (int32_t *)up(NULL, 8);
    CK(nnspk_launch_scalar(2, dx, dy, 1, G.stream));
    int32_t o[2];
    down(o, dy, 8);
    fin();
    *y = o[0];
    *shift = (int8_t)o[1];
}

static void log10_vec_impl(int32_t *out, int32_t *x, int32_t len, int16_t bit_frac_in) /* :53-61 */
{
    if (len <= 0) return;
    begin();
    int32_t *dx = (int32_t *)up(x, (size_t)len * 4);
    int32_t *dy = (int32_t *)up(NULL, (size_t)len * 4);
    CK(nnspk_launch_log10(dy, dx, len, (15 - bit_frac_in) * 0x2688, G.stream));
    down(out, dy, (size_t)len * 4);
    fin();
}

static void my_log10_impl(int32_t *out, int32_t x) { log10_vec(out, &x, 1, 15); } /* :31-50 */

void FeatureClass_construct(FeatureClass *ps, const int32_t *norm_mean, const int32_t *norm_stdR,
                            int8_t qbit_output) /* feature_module.c:12-24 */
{
    stftModule_construct(&ps->state_stftModule);
    ps->pt_norm_mean = norm_mean;
    ps->pt_norm_stdR = norm_stdR;
    ps->num_context = NUM_FEATURE_CONTEXT;
    ps->dim_feat = DIMEMSION_FEATURE;
    ps->qbit_output = qbit_output;
}

static void FeatureClass_setDefault_impl(FeatureClass *ps) /* :26-45 */
{
    stftModule_setDefault(&ps->state_stftModule);
    begin();
    int16_t *dp = (int16_t *)up(ps->normFeatContext + 40, 400);
    int16_t *dt = (int16_t *)up(NULL, 640);
    int32_t *dm = (int32_t *)up(ps->pt_norm_mean, 160);
    int32_t *ds = (int32_t *)up(ps->pt_norm_stdR, 160);
    CK(nnspk_launch_fe_default(dp, dt, dm, ds, 30 - ps->qbit_output, NULL, 1, G.stream));
    int16_t p5[200];
    down(p5, dp, 400);
    fin();
    for (int j = 0; j < NUM_FEATURE_CONTEXT - 1; ++j) memcpy(ps->normFeatContext + 40 * j, p5, 80);
}

static void FeatureClass_execute_impl(FeatureClass *ps, int16_t *input) /* :47-74 */
{
    int16_t tail[320], f5[40];
    memcpy(tail, ps->state_stftModule.dataBuffer + 160, sizeof tail);
    fe_frame(tail, input, ps->pt_norm_mean, ps->pt_norm_stdR, ps->qbit_output, f5, ps->feature, NULL, port_on());
    memmove(ps->normFeatContext, ps->normFeatContext + 40, 200 * 2);
    memcpy(ps->normFeatContext + 200, f5, 80);
    memmove(ps->state_stftModule.dataBuffer, ps->state_stftModule.dataBuffer + 160, 320 * 2);
    memcpy(ps->state_stftModule.dataBuffer + 320, input, 160 * 2);
}

/* ---------------------------------------------------------------------------
 * NNSPClass (nn_speech.c)
 * ------------------------------------------------------------------------- */
int NNSPClass_init(NNSPClass *pt_inst, void *pt_net, void *pt_feat, char nn_id, const int32_t *pt_mean,
                   const int32_t *pt_stdR, int16_t *pt_thresh_prob, int16_t *pt_th_count_trigger)
{ /* :23-55 */
    pt_inst->nn_id = nn_id;
    pt_inst->pt_feat = pt_feat;
    pt_inst->pt_net = pt_net;
    FeatureClass_construct((FeatureClass *)pt_feat, pt_mean, pt_stdR,
                           ((NeuralNetClass *)pt_net)->qbit_input[0]);
    pt_inst->num_dnsmpl = 2;
    pt_inst->pt_thresh_prob = pt_thresh_prob;
    pt_inst->pt_th_count_trigger = pt_th_count_trigger;
    NeuralNetClass_init((NeuralNetClass *)pt_net);
    return 0;
}

static int NNSPClass_reset_impl(NNSPClass *pt_inst) /* :57-72 */
{
    FeatureClass_setDefault((FeatureClass *)pt_inst->pt_feat);
    NeuralNetClass_setDefault((NeuralNetClass *)pt_inst->pt_net);
    pt_inst->slides = 1;
    pt_inst->trigger = 0;
    for (int i = 0; i < DIM_INTENTS; ++i) pt_inst->counts_category[i] = 0;
    for (int i = 0; i < 3; ++i) pt_inst->outputs[i] = 0;
    pt_inst->argmax_last = 0;
    return 0;
}

static void post_pack(const NNSPClass *p, NnPost *q)
{
    memset(q, 0, sizeof *q);
    q->slides = p->slides;
    q->trigger = p->trigger;
    q->argmax_last = p->argmax_last;
    memcpy(q->counts, p->counts_category, sizeof q->counts);
    memcpy(q->outputs, p->outputs, sizeof q->outputs);
}

static void post_unpack(NNSPClass *p, const NnPost *q)
{
    p->slides = (int8_t)q->slides;
    p->trigger = q->trigger;
    p->argmax_last = q->argmax_last;
    memcpy(p->counts_category, q->counts, sizeof q->counts);
    memcpy(p->outputs, q->outputs, sizeof q->outputs);
}

static size_t al16(size_t n) { return (n + 15) & ~(size_t)15; }

/* One frame as a GPU batch of one stream.  Everything the call reads and
 * returns sits in one staging buffer of mapped host memory; one kernel
 * (dropin_kernel) copies the inputs to device memory, runs the front end and
 * the NN, and copies the results back (per frame: one launch and one
 * synchronisation).  NNSP_DROPIN_COPY=1: a pinned buffer with one upload and
 * one download around the launches (round 5 before this; separate small
 * copies from pageable memory made a frame ~160-250 us, bench.py
 * --dropin-latency). */
/* development probe (NNSP_DROPIN_PROBE): host clock, ns */
static long long host_ns(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (long long)ts.tv_sec * 1000000000LL + ts.tv_nsec;
}

/* The resident workers' mailboxes: 64 bytes each below the probe area of the
 * mapped staging; word 0 the request's sequence number, word 1 stop. */
static size_t mbox_off(int k) { return G.hpin_cap - 16 - NNSP_PROBE_BYTES - 64 * (size_t)(k + 1); }
/* worker k's mailbox: host view, device address */
static uint32_t *mbox_host(int k) { return G.dmb ? (uint32_t *)(G.dmb + 64 * (size_t)k) : (uint32_t *)(G.hmap + mbox_off(k)); }
static const uint32_t *mbox_dev(int k)
{
    return G.dmb ? (const uint32_t *)(G.dmb + 64 * (size_t)k) : (const uint32_t *)(G.hmap_dev + mbox_off(k));
}
/* the host's stores to G.dmb (write-combined device memory) drained, in order */
static void dmb_fence(void)
{
    if (G.dmb) __builtin_ia32_sfence();
}

static void worker_stop(int k)
{
    struct dropin_worker *w = &G.W[k];
    if (!w->live) return;
    __atomic_store_n(mbox_host(k) + 1, 1u, __ATOMIC_RELEASE);
    dmb_fence();
    w->live = 0;
    CK(nnspk_sync(w->stream));
}
static void workers_stop(void)
{
    for (int k = 0; k < NNSP_WORKERS; ++k) worker_stop(k);
}
/* at exit: every live worker told to leave (its idle limit would end it too) */
static void workers_atexit(void)
{
    for (int k = 0; k < NNSP_WORKERS; ++k)
        if (G.W[k].live) {
            __atomic_store_n(mbox_host(k) + 1, 1u, __ATOMIC_RELEASE);
            dmb_fence();
        }
}

/* the call (inputs staged, completion word cleared) to the live worker with
 * these arguments, or to a worker launched for them; returns its slot */
static int worker_post(const FeArgs *a, const NnImage *img, const NnRun *r)
{
    static int registered;
    NnRun rc = *r;
    rc.done_seq = 0;
    const long long now = host_ns();
    int k = -1, pick = 0;
    for (int i = 0; i < NNSP_WORKERS; ++i) {
        const struct dropin_worker *w = &G.W[i];
        if (w->live && !memcmp(&w->a, a, sizeof *a) && !memcmp(&w->img, img, sizeof *img) &&
            !memcmp(&w->r, &rc, sizeof rc)) {
            k = i;
            break;
        }
        const struct dropin_worker *p = &G.W[pick];
        if (p->live && (!w->live || w->last < p->last)) pick = i;   /* a free slot, else the least recent */
    }
    /* (a worker idle for half its limit may be leaving: replaced, not posted to) */
    if (k >= 0 && now - G.W[k].last < G.idle_ns / 2) {
        G.W[k].last = now;
        dmb_fence();   /* (the inputs first) */
        __atomic_store_n(mbox_host(k), (uint32_t)r->done_seq, __ATOMIC_RELEASE);
        dmb_fence();
        return k;
    }
    if (k < 0) k = pick;
    worker_stop(k);
    struct dropin_worker *w = &G.W[k];
    if (!w->stream) CK(nnspk_stream_create(&w->stream));
    uint32_t *mb = mbox_host(k);
    mb[1] = 0;
    dmb_fence();
    __atomic_store_n(mb, (uint32_t)r->done_seq, __ATOMIC_RELEASE);
    dmb_fence();
    CK(nnspk_launch_dropin_worker(a, img, r, mbox_dev(k), (uint32_t)r->done_seq, G.idle_ns / 10, w->stream));
    w->a = *a;
    w->img = *img;
    w->r = rc;
    w->live = 1;
    w->last = now;
    if (!registered) registered = atexit(workers_atexit) == 0;
    return k;
}

static int16_t NNSPClass_exec_impl(NNSPClass *pt_inst, int16_t *rawPCM) /* :74-127 */
{
    FeatureClass *fe = (FeatureClass *)pt_inst->pt_feat;
    NeuralNetClass *net = (NeuralNetClass *)pt_inst->pt_net;
    long long hc[5] = {0, 0, 0, 0, 0};   /* NNSP_DROPIN_PROBE: entry, image found, staged, launched, done */
    if (G.probe) hc[0] = host_ns();
    begin();
    /* the tables' bytes are compared with the image's while the call runs: a
     * call that ran on tables since rewritten in place is run again */
    int checked = 0;
    img_node *n = net_image_ex(net, 0, &checked);
restart:
    if (G.probe) hc[1] = host_ns();
    NnImage img = n->im.img;
    img.nn_id = pt_inst->nn_id;
    img.thresh_prob = *pt_inst->pt_thresh_prob;
    img.th_count = *pt_inst->pt_th_count_trigger;
    const int hs = net_hs(net);
    int nls = 0;
    for (int i = 0; i < net->numlayers && i < NN_MAX_LAYERS; ++i) nls += net->net_layer_type[i] == lstm;
    if (nls > NN_MAX_LSTM) nls = NN_MAX_LSTM;
    const size_t rows = (size_t)(nls ? nls : 1);
    /* staging layout: inputs | state in and out | outputs */
    const size_t o_pcm = 0, o_tail = 320, o_mean = o_tail + 640, o_std = o_mean + 160, o_p5 = o_std + 160;
    const size_t o_post = al16(o_p5 + 400), o_h = o_post + al16(sizeof(NnPost)), o_c = o_h + al16(rows * hs * 2);
    const size_t o_feat = o_c + al16(rows * hs * 4), o_log = o_feat + 80, o_trig = o_log + 160;
    /* the completion word sits at a fixed offset past every net's staging:
     * at o_done = total it moved with the net's h/c size, and after a call to a
     * larger net a smaller net's word held that call's state bytes, which could
     * equal the new sequence number by chance (a stale read, no wait) */
    /* (and below it NNSP_PROBE_BYTES of development probes, NNSP_DROPIN_PROBE) */
    const size_t total = al16(o_trig + 2), o_done = G.hpin_cap - 16, o_probe = o_done - NNSP_PROBE_BYTES;
    if (total > mbox_off(NNSP_WORKERS - 1)) fail(NNSP_EUNSUPPORTED, "NNSPClass_exec: staging");
    uint8_t *hp = G.copy ? G.hpin : G.hmap;
    memcpy(hp + o_pcm, rawPCM, 320);
    memcpy(hp + o_tail, fe->state_stftModule.dataBuffer + 160, 640);
    memcpy(hp + o_mean, fe->pt_norm_mean, 160);
    memcpy(hp + o_std, fe->pt_norm_stdR, 160);
    memcpy(hp + o_p5, fe->normFeatContext + 40, 400);
    NnPost ps;
    post_pack(pt_inst, &ps);
    memcpy(hp + o_post, &ps, sizeof ps);
    memset(hp + o_h, 0, o_feat - o_h);
    {
        int l = 0;
        for (int i = 0; i < net->numlayers && l < NN_MAX_LSTM; ++i)
            if (net->net_layer_type[i] == lstm) {
                const int N = net->size_layer[i + 1];
                memcpy(hp + o_h + (size_t)l * hs * 2, net->pt_hstate[i], (size_t)N * 2);
                memcpy(hp + o_c + (size_t)l * hs * 4, net->pt_cstate[i], (size_t)N * 4);
                ++l;
            }
    }
    if (G.probe) hc[2] = host_ns();
    uint8_t *d = (uint8_t *)dscratch(total);
    if (G.copy) CK(nnspk_h2d(d, hp, o_feat, G.stream));
    FeArgs a;
    memset(&a, 0, sizeof a);
    if (!G.copy) { /* (o_feat: a multiple of 16) */
        a.in_src = G.hmap_dev;
        a.in_dst = d;
        a.in_bytes = (int32_t)o_feat;
    }
    a.pcm = (const int16_t *)(d + o_pcm);
    a.tail = (const int16_t *)(d + o_tail);
    a.S = 1; a.T = 1;
    a.mean = (const int32_t *)(d + o_mean);
    a.stdR = (const int32_t *)(d + o_std);
    a.norm_shift = 30 - fe->qbit_output;
    a.feats = (int16_t *)(d + o_feat);
    a.dbg_log = (int32_t *)(d + o_log);
    a.port = port_on();
    if (!G.fetab[a.port]) { /* deriving them in every launch was ~20 us of dependent loads per frame */
        FeArgs ta;
        memset(&ta, 0, sizeof ta);
        ta.mode = FE_MODE_BATCH;
        ta.port = a.port;
        CK(nnspk_build_fe_tables(&G.fetab[a.port], &ta, G.stream));
    }
    a.tb_img = G.fetab[a.port];
    if (G.copy) CK(nnspk_launch_fe(&a, G.stream));
    NnRun r;
    memset(&r, 0, sizeof r);
    r.S = 1; r.T = 1; r.mode = NN_MODE_STREAM; r.nl_run = img.nl;
    r.feats = a.feats;
    r.prev5 = (const int16_t *)(d + o_p5);
    r.hs = hs;
    r.h = (int16_t *)(d + o_h);
    r.c = (int32_t *)(d + o_c);
    r.post = d + o_post;
    r.trig = (int16_t *)(d + o_trig);
    if (!G.copy) { /* (o_post and total: multiples of 16) */
        r.out_src = d + o_post;
        r.out_dst = G.hmap_dev + o_post;
        r.out_bytes = (int32_t)(total - o_post);
        if (G.wait == 2) {
            r.done = (uint32_t *)(G.hmap_dev + o_done);
            r.done_seq = (int32_t)++G.seq;
            /* a value the kernel's store cannot be mistaken for, before the launch */
            __atomic_store_n((uint32_t *)(G.hmap + o_done), ~(uint32_t)r.done_seq, __ATOMIC_RELEASE);
        }
        if (G.probe) r.probe = (long long *)(G.hmap_dev + o_probe);
        if (G.lds) r.st_bytes = (int32_t)total;
    }
    int wk = -1;   /* the resident worker serving the call */
    if (G.copy) {
        CK(nnspk_launch_nn(&img, &r, G.stream));
        CK(nnspk_d2h(hp + o_post, d + o_post, total - o_post, G.stream));
    } else if (G.worker && G.lds && G.wait == 2 && nnspk_dropin_worker_ok(&img, &r)) {
        FeArgs aw = a;
        if (G.dmb && o_feat <= DMB_BYTES - DMB_IN) { /* the inputs where the worker reads them */
            memcpy(G.dmb + DMB_IN, hp, o_feat);
            aw.in_src = G.dmb + DMB_IN;
        }
        wk = worker_post(&aw, &img, &r);
    } else {   /* the front end and the NN in one launch */
        CK(nnspk_launch_dropin(&a, &img, &r, G.lds && G.karg ? hp : NULL, G.stream));
    }
    if (G.probe) hc[3] = host_ns();
    const int stale = !checked && !net_tables_match(net, n);
    checked = 1;
    if (wk >= 0) {
        /* a worker that left before it saw the request (its idle limit): the
         * call in one launch instead, from the same staging */
        if (wait_word_on((volatile uint32_t *)(G.hmap + o_done), (uint32_t)r.done_seq, G.W[wk].stream)) {
            G.W[wk].live = 0;
            CK(nnspk_launch_dropin(&a, &img, &r, G.karg ? hp : NULL, G.stream));
            wait_word((volatile uint32_t *)(G.hmap + o_done), (uint32_t)r.done_seq);
        }
    } else if (!G.copy && G.wait == 2)
        wait_word((volatile uint32_t *)(G.hmap + o_done), (uint32_t)r.done_seq);
    else if (!G.copy && G.wait == 1)
        CK(nnspk_stream_spin(G.stream));
    else
        fin();
    if (stale) { /* (the caller's state is untouched until here) */
        n = net_image(net);
        goto restart;
    }
    memcpy(&ps, hp + o_post, sizeof ps);
    {
        int l = 0;
        for (int i = 0; i < net->numlayers && l < NN_MAX_LSTM; ++i)
            if (net->net_layer_type[i] == lstm) {
                const int N = net->size_layer[i + 1];
                memcpy(net->pt_hstate[i], hp + o_h + (size_t)l * hs * 2, (size_t)N * 2);
                memcpy(net->pt_cstate[i], hp + o_c + (size_t)l * hs * 4, (size_t)N * 4);
                ++l;
            }
    }
    memcpy(fe->feature, hp + o_log, 160);
    memmove(fe->normFeatContext, fe->normFeatContext + 40, 200 * 2);
    memcpy(fe->normFeatContext + 200, hp + o_feat, 80);
    memmove(fe->state_stftModule.dataBuffer, fe->state_stftModule.dataBuffer + 160, 320 * 2);
    memcpy(fe->state_stftModule.dataBuffer + 320, rawPCM, 160 * 2);
    post_unpack(pt_inst, &ps);
    if (G.probe && !G.copy) { /* host phases into the probe area's last longs [88, 93): the kernel wrote its own before */
        hc[4] = host_ns();
        long long *hp_probe = (long long *)(G.hmap + o_probe);
        for (int k = 0; k < 5; ++k) hp_probe[88 + k] = hc[k];
    }
    return pt_inst->trigger;
}

static void my_argmax_impl(int32_t *vec, int len, int16_t *Imax) /* :130-144 */
{
    begin();
    int32_t *dv = (int32_t *)up(vec, (size_t)len * 4);
    int32_t *dy = (int32_t *)up(NULL, 4);
    CK(nnspk_launch_scalar(3, dv, dy, len, G.stream));
    int32_t o;
    down(&o, dy, 4);
    fin();
    *Imax = (int16_t)o;
}

static int32_t scalar1(int op, int32_t x)
{
    begin();
    int32_t *dx = (int32_t *)up(&x, 4);
    int32_t *dy = (int32_t *)up(NULL, 4);
    CK(nnspk_launch_scalar(op, dx, dy, 1, G.stream));
    int32_t o;
    down(&o, dy, 4);
    fin();
    return o;
}
static int32_t ceiling_impl(int32_t input) { return scalar1(0, input); }      /* :229-235 */
static int32_t compute_pwr2_impl(int32_t input) { return scalar1(1, input); } /* :237-258 */

static void post_call(NNSPClass *pt_inst, int32_t *est, int16_t *pt_trigger, int nn_id)
{
    begin();
    NnPost ps;
    post_pack(pt_inst, &ps);
    void *dps = up(&ps, sizeof ps);
    const int n = nn_id == 0 ? 41 : 2;
    int32_t *de = (int32_t *)up(est, (size_t)n * 4);
    CK(nnspk_launch_post(nn_id, *pt_inst->pt_thresh_prob, *pt_inst->pt_th_count_trigger, dps, de,
                         G.stream));
    down(&ps, dps, sizeof ps);
    down(est, de, (size_t)n * 4);
    fin();
    const int16_t keep = pt_inst->trigger;
    post_unpack(pt_inst, &ps);
    pt_inst->trigger = keep;
    *pt_trigger = ps.trigger;
}

static void binary_post_proc_impl(NNSPClass *pt_inst, int32_t *pt_nn_est, int16_t *pt_trigger) /* :191-227 */
{
    post_call(pt_inst, pt_nn_est, pt_trigger, 1);
}

static void s2i_post_proc_impl(NNSPClass *pt_inst, int32_t *pt_nn_est, int16_t *pt_trigger) /* :146-189 */
{
    post_call(pt_inst, pt_nn_est, pt_trigger, 0);
}

/* ---------------------------------------------------------------------------
 * row-block primitives (affine.c:12-407, :492-591; affine_acc32b.c) on the GPU
 * (k_rows: one thread per output row).  Pointer arguments advance exactly as
 * the reference's: the kernel stream by rows * dim_input bytes, the bias by
 * rows (when present), the output by the activation's width (when is_out).
 * ------------------------------------------------------------------------- */
static int row_act(void *(*act)(void *, int32_t *, int), int is_out)
{
    if (!is_out) return 0;
    const int a = nnsp_act_of(act);
    if (a < 0) fprintf(stderr, "libnnsp_mi355x: unsupported activation function pointer\n");
    return a;
}

/* affine_Krows_8x16 (+_acc32b): acc64 accumulators, or int32 ones widened */
static int affine_rows_call(int16_t R, int16_t **pp_output, int8_t **pp_kernel, int16_t **pp_bias,
                            int16_t *input, int16_t K, int16_t qk, int16_t qb, int16_t qi, int64_t *acc64,
                            int32_t *acc32, int8_t is_out, void *(*act)(void *, int32_t *, int))
{
    if (R < 1 || R > 4 || K < 0) return -1;
    const int a_t = row_act(act, is_out);
    if (a_t < 0) return -1;
    begin();
    RowArgs a;
    memset(&a, 0, sizeof a);
    a.mode = ROWS_AFFINE;
    a.rows = R;
    a.K = K;
    a.qk = qk; a.qb = qb; a.qi = qi;
    a.acc32 = acc32 != NULL;
    a.is_out = is_out;
    a.act = a_t;
    a.port = port_on();
    int64_t acc[4];
    for (int i = 0; i < R; ++i) acc[i] = acc32 ? (int64_t)acc32[i] : acc64[i];
    a.w = (const int8_t *)up(*pp_kernel, (size_t)R * K);
    a.b = *pp_bias ? (const int16_t *)up(*pp_bias, (size_t)R * 2) : NULL;
    a.x = (const int16_t *)up(input, (size_t)K * 2);
    a.acc = (int64_t *)up(acc, (size_t)R * 8);
    const size_t ob = (size_t)R * (a_t == 3 ? 4 : 2);
    if (is_out) a.out = up(NULL, ob);
    CK(nnspk_launch_rows(&a, G.stream));
    down(acc, a.acc, (size_t)R * 8);
    if (is_out) down(*pp_output, a.out, ob);
    fin();
    for (int i = 0; i < R; ++i) {
        if (acc32) acc32[i] = (int32_t)acc[i];
        else acc64[i] = acc[i];
    }
    *pp_kernel += (size_t)R * K;
    if (*pp_bias) *pp_bias += R;
    if (is_out) *pp_output = (int16_t *)((char *)*pp_output + ob);
    return 0;
}

static int affine_Krows_8x16_impl(int16_t dim_output, int16_t **pp_output, int8_t **pp_kernel, int16_t **pp_bias,
                      int16_t *input, int16_t dim_input, int16_t qbit_kernel, int16_t qbit_bias,
                      int16_t qbit_input, int64_t *pt_accum, int8_t is_out,
                      void *(*act)(void *, int32_t *, int)) /* affine.c:12-259 */
{
    return affine_rows_call(dim_output, pp_output, pp_kernel, pp_bias, input, dim_input, qbit_kernel, qbit_bias,
                            qbit_input, pt_accum, NULL, is_out, act);
}

static int affine_Krows_8x16_acc32b_impl(int16_t dim_output, int16_t **pp_output, int8_t **pp_kernel, int16_t **pp_bias,
                             int16_t *input, int16_t dim_input, int16_t qbit_kernel, int16_t qbit_bias,
                             int16_t qbit_input, int32_t *pt_accum, int8_t is_out,
                             void *(*act)(void *, int32_t *, int)) /* affine_acc32b.c:12-260 */
{
    return affine_rows_call(dim_output, pp_output, pp_kernel, pp_bias, input, dim_input, qbit_kernel, qbit_bias,
                            qbit_input, NULL, pt_accum, is_out, act);
}

/* rc_Krows_8x16 (one group of <= 4 rows) and rc_8x16 (a whole layer) */
static int rc_rows_call(int rows, int16_t *p_output, const int8_t *w, const int8_t *wr, const int16_t *bias,
                        int16_t *input, int16_t *input_rec, int K, int Kr, int qk, int qb, int qi, int qir,
                        int acc32, void *(*act)(void *, int32_t *, int), size_t *out_bytes)
{
    const int a_t = row_act(act, 1);
    if (a_t < 0 || rows < 1 || K < 0 || Kr < 0) return -1;
    begin();
    RowArgs a;
    memset(&a, 0, sizeof a);
    a.mode = ROWS_RC;
    a.rows = rows;
    a.K = K;
    a.Kr = Kr;
    a.qk = qk; a.qb = qb; a.qi = qi; a.qir = qir;
    a.acc32 = acc32;
    a.is_out = 1;
    a.act = a_t;
    a.port = port_on();
    a.w = (const int8_t *)up(w, (size_t)rows * K);
    a.wr = (const int8_t *)up(wr, (size_t)rows * Kr);
    a.b = bias ? (const int16_t *)up(bias, (size_t)rows * 2) : NULL;
    a.x = (const int16_t *)up(input, (size_t)K * 2);
    a.xr = (const int16_t *)up(input_rec, (size_t)Kr * 2);
    *out_bytes = (size_t)rows * (a_t == 3 ? 4 : 2);
    a.out = up(NULL, *out_bytes);
    CK(nnspk_launch_rows(&a, G.stream));
    down(p_output, a.out, *out_bytes);
    fin();
    return 0;
}

static int rc_krows(int16_t R, int16_t **pp_output, int8_t **pp_kernel, int8_t **pp_kernel_rec, int16_t **pp_bias,
                    int16_t *input, int16_t *input_rec, int16_t K, int16_t Kr, int16_t qk, int16_t qb, int16_t qi,
                    int16_t qir, int acc32, void *(*act)(void *, int32_t *, int))
{
    if (R < 1 || R > 4) return -1;
    size_t ob = 0;
    if (rc_rows_call(R, *pp_output, *pp_kernel, *pp_kernel_rec, *pp_bias, input, input_rec, K, Kr, qk, qb, qi, qir,
                     acc32, act, &ob))
        return -1;
    *pp_output = (int16_t *)((char *)*pp_output + ob);
    *pp_kernel += (size_t)R * K;
    *pp_kernel_rec += (size_t)R * Kr;
    if (*pp_bias) *pp_bias += R;
    return 0;
}

static int rc_Krows_8x16_impl(int16_t dim_output, int16_t **pp_output, int8_t **pp_kernel, int8_t **pp_kernel_rec,
                  int16_t **pp_bias, int16_t *input, int16_t *input_rec, int16_t dim_input, int16_t dim_input_rec,
                  int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input, int16_t qbit_input_rec,
                  void *(*act)(void *, int32_t *, int)) /* affine.c:348-407 */
{
    return rc_krows(dim_output, pp_output, pp_kernel, pp_kernel_rec, pp_bias, input, input_rec, dim_input,
                    dim_input_rec, qbit_kernel, qbit_bias, qbit_input, qbit_input_rec, 0, act);
}

static int rc_Krows_8x16_acc32b_impl(int16_t dim_output, int16_t **pp_output, int8_t **pp_kernel, int8_t **pp_kernel_rec,
                         int16_t **pp_bias, int16_t *input, int16_t *input_rec, int16_t dim_input,
                         int16_t dim_input_rec, int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input,
                         int16_t qbit_input_rec, void *(*act)(void *, int32_t *, int)) /* affine_acc32b.c:349-408 */
{
    return rc_krows(dim_output, pp_output, pp_kernel, pp_kernel_rec, pp_bias, input, input_rec, dim_input,
                    dim_input_rec, qbit_kernel, qbit_bias, qbit_input, qbit_input_rec, 1, act);
}

static int rc_8x16_impl(int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias, int16_t *input,
            int16_t *input_rec, int16_t dim_output, int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel,
            int16_t qbit_bias, int16_t qbit_input, int16_t qbit_input_rec, ACTIVATION_TYPE act_type,
            void *(*act)(void *, int32_t *, int)) /* affine.c:492-563 */
{
    (void)act_type;
    size_t ob = 0;
    return rc_rows_call(dim_output, p_output, p_kernel, p_kernel_rec, p_bias, input, input_rec, dim_input,
                        dim_input_rec, qbit_kernel, qbit_bias, qbit_input, qbit_input_rec, 0, act, &ob);
}

static int rc_8x16_acc32b_impl(int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias, int16_t *input,
                   int16_t *input_rec, int16_t dim_output, int16_t dim_input, int16_t dim_input_rec,
                   int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input, int16_t qbit_input_rec,
                   ACTIVATION_TYPE act_type, void *(*act)(void *, int32_t *, int)) /* affine_acc32b.c:493-564 */
{
    (void)act_type;
    size_t ob = 0;
    return rc_rows_call(dim_output, p_output, p_kernel, p_kernel_rec, p_bias, input, input_rec, dim_input,
                        dim_input_rec, qbit_kernel, qbit_bias, qbit_input, qbit_input_rec, 1, act, &ob);
}

static void shift_call(void *x, int shift, int len, int acc32)
{
    if (len <= 0 || shift == 0) return;
    begin();
    const size_t nb = (size_t)len * (acc32 ? 4 : 8);
    void *d = up(x, nb);
    CK(nnspk_launch_shift(d, shift, len, acc32, G.stream));
    down(x, d, nb);
    fin();
}
static void shift_64b_impl(int64_t *x, int8_t shift, int len) { shift_call(x, shift, len, 0); } /* affine.c:565-591 */
static void shift_32b_impl(int32_t *x, int8_t shift, int len) { shift_call(x, shift, len, 1); } /* affine_acc32b.c:566-592 */

/* ---------------------------------------------------------------------------
 * public entry points: a HIP or allocation failure inside any of them unwinds
 * to the outermost one (longjmp from CK), which returns with its outputs
 * untouched; the error stays readable through nnsp_legacy_status() /
 * nnsp_strerror() (the reference has no error channel: its functions return
 * 0 or void).  Nested entry points (NNSPClass_reset -> FeatureClass_setDefault)
 * share the outermost jump target.
 * ------------------------------------------------------------------------- */
/* The public entry points: the outermost one sets fail()'s longjmp target
 * and returns onfail (void: nothing) when a GPU step fails inside it. */
#define LEGACY_ENTRY(ret, name, params, args, onfail) \
    ret name params                                   \
    {                                                 \
        if (G.depth++ == 0) {                         \
            if (setjmp(G.jb)) {                       \
                G.depth = 0;                          \
                return onfail;                        \
            }                                         \
        }                                             \
        ret r_ = name##_impl args;                    \
        --G.depth;                                    \
        return r_;                                    \
    }
#define LEGACY_ENTRY_VOID(name, params, args) \
    void name params                          \
    {                                         \
        if (G.depth++ == 0) {                 \
            if (setjmp(G.jb)) {               \
                G.depth = 0;                  \
                return;                       \
            }                                 \
        }                                     \
        name##_impl args;                     \
        --G.depth;                            \
    }

LEGACY_ENTRY(void *, relu6_fix, (int16_t *y, int32_t *x, int len), (y, x, len), NULL)

LEGACY_ENTRY(void *, tanh_fix, (int16_t *y, int32_t *x, int len), (y, x, len), NULL)

LEGACY_ENTRY(void *, sigmoid_fix, (int16_t *y, int32_t *x, int len), (y, x, len), NULL)

LEGACY_ENTRY(void *, linear_fix, (int32_t *y, int32_t *x, int len), (y, x, len), NULL)

LEGACY_ENTRY(int, fc_8x16, (int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias, int16_t *input, int16_t *input_rec, int32_t *c_state, int16_t dim_output, int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input, int16_t qbit_input_rec, ACTIVATION_TYPE act_type, void *(*act)(void *, int32_t *, int)), (p_output, p_kernel, p_kernel_rec, p_bias, input, input_rec, c_state, dim_output, dim_input, dim_input_rec, qbit_kernel, qbit_bias, qbit_input, qbit_input_rec, act_type, act), G.sticky)

LEGACY_ENTRY(int, fc_8x16_acc32b, (int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias, int16_t *input, int16_t *input_rec, int32_t *c_state, int16_t dim_output, int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input, int16_t qbit_input_rec, ACTIVATION_TYPE act_type, void *(*act)(void *, int32_t *, int)), (p_output, p_kernel, p_kernel_rec, p_bias, input, input_rec, c_state, dim_output, dim_input, dim_input_rec, qbit_kernel, qbit_bias, qbit_input, qbit_input_rec, act_type, act), G.sticky)

LEGACY_ENTRY(int, lstm_8x16, (int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias, int16_t *input, int16_t *h_state, int32_t *c_state, int16_t dim_output, int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input, int16_t qbit_input_rec, ACTIVATION_TYPE act_type, void *(*act)(void *, int32_t *, int)), (p_output, p_kernel, p_kernel_rec, p_bias, input, h_state, c_state, dim_output, dim_input, dim_input_rec, qbit_kernel, qbit_bias, qbit_input, qbit_input_rec, act_type, act), G.sticky)

LEGACY_ENTRY(int, lstm_8x16_acc32b, (int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias, int16_t *input, int16_t *h_state, int32_t *c_state, int16_t dim_output, int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input, int16_t qbit_input_rec, ACTIVATION_TYPE act_type, void *(*act)(void *, int32_t *, int)), (p_output, p_kernel, p_kernel_rec, p_bias, input, h_state, c_state, dim_output, dim_input, dim_input_rec, qbit_kernel, qbit_bias, qbit_input, qbit_input_rec, act_type, act), G.sticky)

LEGACY_ENTRY_VOID(NeuralNetClass_exe, (NeuralNetClass *pt_inst, int16_t *input, int32_t *output, int8_t debug_layer), (pt_inst, input, output, debug_layer))

LEGACY_ENTRY_VOID(arm_fft_exec, (int32_t *y, int32_t *x), (y, x))

LEGACY_ENTRY(int, stftModule_analyze_arm, (void *ps_, int16_t *x, int32_t *y), (ps_, x, y), G.sticky)

LEGACY_ENTRY_VOID(spec2pspec_arm, (int32_t *y, int32_t *x, int len), (y, x, len))

LEGACY_ENTRY(int, stftModule_analyze, (stftModule *ps, int16_t *x, int32_t *y), (ps, x, y), G.sticky)

LEGACY_ENTRY_VOID(spec2pspec, (int32_t *y, int32_t *x, int len), (y, x, len))

LEGACY_ENTRY_VOID(rfft, (int num_rfft, int32_t *input, void *output), (num_rfft, input, output))

LEGACY_ENTRY_VOID(fft, (int exp_nfft, void *input, void *output), (exp_nfft, input, output))

LEGACY_ENTRY_VOID(complex32_copy, (COMPLEX32 *dst, COMPLEX32 *src), (dst, src))
LEGACY_ENTRY_VOID(complex32_affine, (COMPLEX32 *out, COMPLEX32 *Mat, COMPLEX32 *input, int shift_r, int len),
                  (out, Mat, input, shift_r, len))
LEGACY_ENTRY_VOID(complex32_interprod, (COMPLEX32 *out, COMPLEX32 *arry1, COMPLEX32 *arry2, int shift_r, int len),
                  (out, arry1, arry2, shift_r, len))
LEGACY_ENTRY_VOID(complex32_complex16_elmtprod, (COMPLEX32 *out, COMPLEX32 *arry1, COMPLEX16 *arry2, int len),
                  (out, arry1, arry2, len))
LEGACY_ENTRY_VOID(complex32_add, (COMPLEX32 *out, COMPLEX32 *addr1, COMPLEX32 *addr2), (out, addr1, addr2))
LEGACY_ENTRY_VOID(complexArry32_add, (COMPLEX32 *out, COMPLEX32 *addr1, COMPLEX32 *addr2, int len),
                  (out, addr1, addr2, len))
LEGACY_ENTRY_VOID(complex32_neg, (COMPLEX32 *out, COMPLEX32 *in), (out, in))
LEGACY_ENTRY_VOID(complex32_sub, (COMPLEX32 *out, COMPLEX32 *a, COMPLEX32 *b), (out, a, b))
LEGACY_ENTRY_VOID(complex32_mul, (COMPLEX32 *out, COMPLEX32 *addr1, COMPLEX32 *addr2), (out, addr1, addr2))
LEGACY_ENTRY_VOID(complex32_init, (COMPLEX32 *inst, int32_t real, int32_t imag), (inst, real, imag))
LEGACY_ENTRY_VOID(complex32_real2cmplx, (COMPLEX32 *inst, int32_t real), (inst, real))
LEGACY_ENTRY_VOID(complexArry32_real2cmplx, (COMPLEX32 *inst, int32_t *real, int32_t len), (inst, real, len))
LEGACY_ENTRY_VOID(complexArry32_init, (COMPLEX32 *inst, int32_t *real, int32_t *imag, int len), (inst, real, imag, len))

/* complex.c:174-184 (AMBIQ_NNSP_DEBUG builds): host-side text output only */
void complexArry32_print(COMPLEX32 *inst, int len)
{
    for (int i = 0; i < len; i++) printf("%d: (%d, %d)\n", i, inst[i].real, inst[i].imag);
}

LEGACY_ENTRY_VOID(melSpecProc, (int32_t *specs, int32_t *melSpecs), (specs, melSpecs))

LEGACY_ENTRY_VOID(norm_oneTwo, (int32_t x, int32_t *y, int8_t *shift), (x, y, shift))

LEGACY_ENTRY_VOID(log10_vec, (int32_t *out, int32_t *x, int32_t len, int16_t bit_frac_in), (out, x, len, bit_frac_in))

LEGACY_ENTRY_VOID(my_log10, (int32_t *out, int32_t x), (out, x))

LEGACY_ENTRY_VOID(FeatureClass_setDefault, (FeatureClass *ps), (ps))

LEGACY_ENTRY_VOID(FeatureClass_execute, (FeatureClass *ps, int16_t *input), (ps, input))

LEGACY_ENTRY(int, NNSPClass_reset, (NNSPClass *pt_inst), (pt_inst), G.sticky)

LEGACY_ENTRY(int16_t, NNSPClass_exec, (NNSPClass *pt_inst, int16_t *rawPCM), (pt_inst, rawPCM), 0)

LEGACY_ENTRY_VOID(my_argmax, (int32_t *vec, int len, int16_t *Imax), (vec, len, Imax))

LEGACY_ENTRY(int32_t, ceiling, (int32_t input), (input), 0)

LEGACY_ENTRY(int32_t, compute_pwr2, (int32_t input), (input), 0)

LEGACY_ENTRY_VOID(binary_post_proc, (NNSPClass *pt_inst, int32_t *pt_nn_est, int16_t *pt_trigger), (pt_inst, pt_nn_est, pt_trigger))

LEGACY_ENTRY_VOID(s2i_post_proc, (NNSPClass *pt_inst, int32_t *pt_nn_est, int16_t *pt_trigger), (pt_inst, pt_nn_est, pt_trigger))

LEGACY_ENTRY(int, affine_Krows_8x16, (int16_t dim_output, int16_t **pp_output, int8_t **pp_kernel, int16_t **pp_bias, int16_t *input, int16_t dim_input, int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input, int64_t *pt_accum, int8_t is_out, void *(*act)(void *, int32_t *, int)), (dim_output, pp_output, pp_kernel, pp_bias, input, dim_input, qbit_kernel, qbit_bias, qbit_input, pt_accum, is_out, act), G.sticky)

LEGACY_ENTRY(int, affine_Krows_8x16_acc32b, (int16_t dim_output, int16_t **pp_output, int8_t **pp_kernel, int16_t **pp_bias, int16_t *input, int16_t dim_input, int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input, int32_t *pt_accum, int8_t is_out, void *(*act)(void *, int32_t *, int)), (dim_output, pp_output, pp_kernel, pp_bias, input, dim_input, qbit_kernel, qbit_bias, qbit_input, pt_accum, is_out, act), G.sticky)

LEGACY_ENTRY(int, rc_Krows_8x16, (int16_t dim_output, int16_t **pp_output, int8_t **pp_kernel, int8_t **pp_kernel_rec, int16_t **pp_bias, int16_t *input, int16_t *input_rec, int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input, int16_t qbit_input_rec, void *(*act)(void *, int32_t *, int)), (dim_output, pp_output, pp_kernel, pp_kernel_rec, pp_bias, input, input_rec, dim_input, dim_input_rec, qbit_kernel, qbit_bias, qbit_input, qbit_input_rec, act), G.sticky)

LEGACY_ENTRY(int, rc_Krows_8x16_acc32b, (int16_t dim_output, int16_t **pp_output, int8_t **pp_kernel, int8_t **pp_kernel_rec, int16_t **pp_bias, int16_t *input, int16_t *input_rec, int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input, int16_t qbit_input_rec, void *(*act)(void *, int32_t *, int)), (dim_output, pp_output, pp_kernel, pp_kernel_rec, pp_bias, input, input_rec, dim_input, dim_input_rec, qbit_kernel, qbit_bias, qbit_input, qbit_input_rec, act), G.sticky)

LEGACY_ENTRY(int, rc_8x16, (int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias, int16_t *input, int16_t *input_rec, int16_t dim_output, int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input, int16_t qbit_input_rec, ACTIVATION_TYPE act_type, void *(*act)(void *, int32_t *, int)), (p_output, p_kernel, p_kernel_rec, p_bias, input, input_rec, dim_output, dim_input, dim_input_rec, qbit_kernel, qbit_bias, qbit_input, qbit_input_rec, act_type, act), G.sticky)

LEGACY_ENTRY(int, rc_8x16_acc32b, (int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias, int16_t *input, int16_t *input_rec, int16_t dim_output, int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input, int16_t qbit_input_rec, ACTIVATION_TYPE act_type, void *(*act)(void *, int32_t *, int)), (p_output, p_kernel, p_kernel_rec, p_bias, input, input_rec, dim_output, dim_input, dim_input_rec, qbit_kernel, qbit_bias, qbit_input, qbit_input_rec, act_type, act), G.sticky)

LEGACY_ENTRY_VOID(shift_64b, (int64_t *x, int8_t shift, int len), (x, shift, len))

LEGACY_ENTRY_VOID(shift_32b, (int32_t *x, int8_t shift, int len), (x, shift, len))
