/*
 * nnsp_image.c -- NeuralNetClass -> device image.
 *
 * Reads a reference-format NeuralNetClass (neural_nets.h:15-32): layer types,
 * sizes, qbits, the layer/activation function pointers (to tell the acc32
 * variants and activations apart) and the interleaved int8 weight streams of
 * def_nn*.c.  De-interleaves the CMSIS-NN order the ARM path walks
 * (affine.c:80-184; LSTM gate grouping lstm.c:48-124) and re-tiles every
 * matrix into 1 KiB MFMA A-fragments for v_mfma_i32_16x16x64_i8:
 * fragment (rt, kt), lane l, byte j = W[16*rt + (l & 15)][64*kt + 16*(l >> 4) + j].
 * LSTM rows are permuted so that a row tile holds 4 units x 4 gates
 * (physical row 16*rt + 4*q + g = gate g of unit 4*rt + q).
 */
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nnsp_host.h"

static char g_err[256];

void nnsp_set_error(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

const char *nnsp_last_error(void) { return g_err; }

int nnsp_act_of(void *(*fn)(void *, int32_t *, int))
{
    if (fn == (void *(*)(void *, int32_t *, int))relu6_fix) return 0;
    if (fn == (void *(*)(void *, int32_t *, int))tanh_fix) return 1;
    if (fn == (void *(*)(void *, int32_t *, int))sigmoid_fix) return 2;
    if (fn == (void *(*)(void *, int32_t *, int))linear_fix) return 3;
    return -1;
}

int nnsp_describe_net(const NeuralNetClass *net, nnsp_layer_desc *L, int *nl, int *out_linear)
{
    if (!net || net->numlayers <= 0 || net->numlayers > NN_MAX_LAYERS) {
        nnsp_set_error("numlayers out of range");
        return NNSP_EINVAL;
    }
    *nl = net->numlayers;
    for (int i = 0; i < net->numlayers; ++i) {
        nnsp_layer_desc *d = &L[i];
        memset(d, 0, sizeof *d);
        int *(*lf)() = net->layer_func[i];
        if (lf == (int *(*)())fc_8x16 || lf == (int *(*)())fc_8x16_acc32b) {
            d->type = NN_FC;
            d->acc32 = lf == (int *(*)())fc_8x16_acc32b;
        } else if (lf == (int *(*)())lstm_8x16 || lf == (int *(*)())lstm_8x16_acc32b) {
            d->type = NN_LSTM;
            d->acc32 = lf == (int *(*)())lstm_8x16_acc32b;
        } else {
            nnsp_set_error("layer %d: layer_func is not fc_8x16/lstm_8x16(_acc32b)", i);
            return NNSP_EUNSUPPORTED;
        }
        if ((d->type == NN_LSTM) != (net->net_layer_type[i] == lstm)) {
            nnsp_set_error("layer %d: layer_func disagrees with net_layer_type", i);
            return NNSP_EINVAL;
        }
        d->K = net->size_layer[i];
        d->N = net->size_layer[i + 1];
        d->qk = net->qbit_kernel[i];
        d->qb = net->qbit_bias[i];
        d->qi = net->qbit_input[i];
        d->qir = (i + 1 < 10) ? net->qbit_input[i + 1] : 0; /* neural_nets.c:108 */
        d->W = net->pt_kernel[i];
        d->Wr = net->pt_kernel_rec[i];
        d->B = net->pt_bias[i];
        if (d->type == NN_FC) {
            d->act = nnsp_act_of(net->act_func[i]);
            if (d->act < 0) {
                nnsp_set_error("layer %d: unsupported activation function", i);
                return NNSP_EUNSUPPORTED;
            }
            const int want_lin = net->activation_type[i] == linear;
            if (want_lin != (d->act == 3)) {
                nnsp_set_error("layer %d: act_func disagrees with activation_type", i);
                return NNSP_EINVAL;
            }
        } else {
            d->act = 1;
            if (!d->Wr) {
                nnsp_set_error("layer %d: LSTM without kernel_rec", i);
                return NNSP_EINVAL;
            }
        }
    }
    *out_linear = net->activation_type[net->numlayers - 1] == linear;
    return 0;
}

/* Walk one affine_Krows block of R rows x K columns (affine.c:74-184):
 * call put(row, col, byte) in stream order; returns bytes consumed. */
static size_t walk_block(const int8_t *w, int R, int K, int8_t *dst, int dst_ld, int row0)
{
    size_t o = 0;
    for (int p = 0; p < K / 2; ++p) {
        const int c0 = 2 * p, c1 = 2 * p + 1;
#define PUT(r, c) dst[(size_t)(row0 + (r)) * dst_ld + (c)] = w[o++]
        if (R == 4) {
            PUT(0, c0); PUT(1, c0); PUT(0, c1); PUT(1, c1);
            PUT(2, c0); PUT(3, c0); PUT(2, c1); PUT(3, c1);
        } else if (R == 3) {
            PUT(0, c0); PUT(1, c0); PUT(0, c1); PUT(1, c1); PUT(2, c0); PUT(2, c1);
        } else if (R == 2) {
            PUT(0, c0); PUT(1, c0); PUT(0, c1); PUT(1, c1);
        } else {
            PUT(0, c0); PUT(0, c1);
        }
    }
    if (K & 1)
        for (int r = 0; r < R; ++r) PUT(r, K - 1);
#undef PUT
    return o;
}

/* The ARM_OPTIMIZED=0 build's walk of one R-row block (affine.c:261-346):
 * per column pair, per row, the pair's two bytes; an odd K's last column per
 * row after the pairs. */
static size_t walk_block_portable(const int8_t *w, int R, int K, int8_t *dst, int dst_ld, int row0)
{
    size_t o = 0;
    for (int p = 0; p < K / 2; ++p)
        for (int r = 0; r < R; ++r) {
            dst[(size_t)(row0 + r) * dst_ld + 2 * p] = w[o++];
            dst[(size_t)(row0 + r) * dst_ld + 2 * p + 1] = w[o++];
        }
    if (K & 1)
        for (int r = 0; r < R; ++r) dst[(size_t)(row0 + r) * dst_ld + K - 1] = w[o++];
    return o;
}

static size_t walk(int portable, const int8_t *w, int R, int K, int8_t *dst, int dst_ld, int row0)
{
    return portable ? walk_block_portable(w, R, K, dst, dst_ld, row0) : walk_block(w, R, K, dst, dst_ld, row0);
}

/* natural [N][K] from an fc_8x16 stream */
static void unpack_fc(const int8_t *w, int N, int K, int8_t *dst, int portable)
{
    for (int r0 = 0; r0 < N; r0 += 4) {
        const int R = N - r0 < 4 ? N - r0 : 4;
        w += walk(portable, w, R, K, dst, K, r0);
    }
}

/* natural gate-major [4N][K] (rows g*N + u) from an lstm_8x16 stream */
static void unpack_lstm(const int8_t *w, int N, int K, int8_t *dst, int portable)
{
    for (int u0 = 0; u0 < N; u0 += 4) {
        const int R = N - u0 < 4 ? N - u0 : 4;
        for (int g = 0; g < 4; ++g) w += walk(portable, w, R, K, dst, K, g * N + u0);
    }
}

/* The accumulator scale qs of an affine_Krows call with a bias (affine.c).
 * Shipped build: max(qin + qk, 15), and the align shift is dead (T1), so the
 * sums stay at Q(qin + qk) while the bias is aligned to qs.  Portable build:
 * the sums are shifted left by 15 - (qin + qk) (clamped) before the bias is
 * added (affine.c:311-313).  The engine's epilogue is bias-then-shift, so the
 * portable form is run as qs = qin + qk: (s + (b << (qs - qb))) << L equals
 * clamp(s << L) + (b << (15 - qb)) exactly when qb <= qs and no clamp can bind
 * -- checked against the worst case |sum| of every row (bound). */
static long long sum_bound(const nnsp_layer_desc *d, int bias_sh);
static int bias_qs(const nnsp_layer_desc *d, int qin, int layer, int *qs)
{
    const int q = qin + d->qk;
    *qs = q > 15 ? q : 15;
    if (!d->portable || q >= 15) return 0;
    const int L = 15 - q;
    const long long bound = sum_bound(d, q - d->qb);
    if (bound < 0) return NNSP_ENOMEM;
    const long long lim = d->acc32 ? (1LL << (31 - L)) : (1LL << 62 >> (L - 1));
    if (d->qb > q || bound >= lim) {
        nnsp_set_error("layer %d: portable align shift %d with qbit_bias %d / sum bound %lld not exactly "
                       "representable", layer, L, d->qb, bound);
        return NNSP_EUNSUPPORTED;
    }
    *qs = q;
    return 0;
}

/* max over rows of |W x| (LSTM: the x part after its qir - qi shift, plus
 * |Wr h|) + |b << bias_sh| for any int16 inputs: the layer's worst-case
 * accumulator (-1: out of memory) */
static void unpack_lstm_bias(const int16_t *b, int N, int16_t *dst);
static long long sum_bound(const nnsp_layer_desc *d, int bias_sh)
{
    const int lstm = d->type == NN_LSTM;
    const int rows = lstm ? 4 * d->N : d->N;
    int8_t *nat = (int8_t *)calloc((size_t)rows * d->K, 1);
    int8_t *natr = lstm ? (int8_t *)calloc((size_t)rows * d->N, 1) : NULL;
    int16_t *bn = (int16_t *)calloc((size_t)rows, sizeof(int16_t));
    long long best = -1;
    if (!nat || !bn || (lstm && !natr)) goto out;
    if (lstm) {
        unpack_lstm(d->W, d->N, d->K, nat, d->portable);
        unpack_lstm(d->Wr, d->N, d->N, natr, d->portable);
        if (d->B) unpack_lstm_bias(d->B, d->N, bn);
    } else {
        unpack_fc(d->W, d->N, d->K, nat, d->portable);
        if (d->B) memcpy(bn, d->B, (size_t)rows * sizeof(int16_t));
    }
    best = 0;
    for (int r = 0; r < rows; ++r) {
        long long sx = 0, sr = 0;
        for (int k = 0; k < d->K; ++k) sx += abs(nat[(size_t)r * d->K + k]);
        if (lstm)
            for (int k = 0; k < d->N; ++k) sr += abs(natr[(size_t)r * d->N + k]);
        long long v = sx * 32768;
        if (lstm) {
            const int xs = d->qir - d->qi;
            v = xs >= 0 ? (xs < 24 ? v << xs : (1LL << 62)) : v >> -xs;
            v += sr * 32768;
        }
        v += (long long)abs(bn[r]) << (bias_sh > 0 ? bias_sh : 0);
        if (v > best) best = v;
    }
out:
    free(nat);
    free(natr);
    free(bn);
    return best;
}

static void unpack_lstm_bias(const int16_t *b, int N, int16_t *dst)
{
    for (int u0 = 0; u0 < N; u0 += 4) {
        const int R = N - u0 < 4 ? N - u0 : 4;
        for (int g = 0; g < 4; ++g)
            for (int r = 0; r < R; ++r) dst[g * N + u0 + r] = *b++;
    }
}

/* physical (re-tiled) row -> natural row, -1 = padding */
static int lstm_row(int p, int N)
{
    const int rt = p / 16, r = p % 16, q = r / 4, g = r % 4, u = 4 * rt + q;
    return u < N ? g * N + u : -1;
}

static void put_frags(uint8_t *A, const int8_t *nat, int K, int nrt, int nkt, int N, int lstm)
{
    for (int rt = 0; rt < nrt; ++rt)
        for (int kt = 0; kt < nkt; ++kt)
            for (int l = 0; l < 64; ++l)
                for (int j = 0; j < 16; ++j) {
                    const int p = 16 * rt + (l & 15), k = 64 * kt + 16 * (l >> 4) + j;
                    const int row = lstm ? lstm_row(p, N) : (p < N ? p : -1);
                    const int8_t v = (row >= 0 && k < K) ? nat[(size_t)row * K + k] : 0;
                    A[((size_t)(rt * nkt + kt) * 64 + l) * 16 + j] = (uint8_t)v;
                }
}

static int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

int nnsp_image_build(nnsp_image *im, const nnsp_layer_desc *L, int nl, int nn_id,
                     int thresh_prob, int th_count, int direct)
{
    memset(im, 0, sizeof *im);
    NnImage *g = &im->img;
    g->nl = nl;
    g->nn_id = nn_id;
    g->thresh_prob = thresh_prob;
    g->th_count = th_count;
    size_t a_bytes = 0;
    int rows_total = 0, n_lstm = 0;
    for (int i = 0; i < nl; ++i) {
        const nnsp_layer_desc *d = &L[i];
        NnLayer *y = &g->L[i];
        /* the reference runs any stack whose widths fit its 300-element
         * int16 activation buffers (neural_nets.c:9-10); a linear layer
         * writes int32, 150 of them */
        const int lin = d->type == NN_FC && d->act == 3;
        if (d->K <= 0 || d->N <= 0 || d->K > NN_MAX_WIDTH || d->N > (lin ? NN_MAX_LIN : NN_MAX_WIDTH)) {
            nnsp_set_error("layer %d: width %d->%d outside the reference's activation buffers (1..%d int16, "
                           "%d int32 for a linear layer)", i, d->K, d->N, NN_MAX_WIDTH, NN_MAX_LIN);
            return NNSP_EUNSUPPORTED;
        }
        if (i > 0 && d->K != L[i - 1].N) {
            nnsp_set_error("layer %d: input width %d != previous output %d", i, d->K, L[i - 1].N);
            return NNSP_EINVAL;
        }
        y->type = d->type;
        y->K = d->K;
        y->N = d->N;
        y->act = d->act;
        y->nkt = (d->K + 63) / 64;
        y->has_bias = d->B != NULL;
        y->acc32 = d->acc32;
        y->ep_off = rows_total;
        y->a_off = (int64_t)a_bytes;
        if (d->type == NN_LSTM) {
            if (n_lstm >= NN_MAX_LSTM) {
                nnsp_set_error("layer %d: more than %d LSTM layers", i, NN_MAX_LSTM);
                return NNSP_EUNSUPPORTED;
            }
            g->lstm_n[n_lstm++] = d->N;
            y->nrt = (d->N + 3) / 4;
            y->rows = 16 * y->nrt;
            y->nkt_r = (d->N + 63) / 64;
            y->ar_off = (int64_t)(a_bytes + (size_t)y->nrt * y->nkt * 1024);
            a_bytes += (size_t)y->nrt * (y->nkt + y->nkt_r) * 1024;
            const int qs1 = d->qi + d->qk; /* first rc half: no bias */
            (void)qs1;
            y->xs_sh = d->qir - d->qi;
            int qs2 = d->qir + d->qk;
            if (y->has_bias) {
                const int e = bias_qs(d, d->qir, i, &qs2);
                if (e) return e;
            }
            y->bias_sh = qs2 - d->qb;
            y->out_sh = 15 - qs2;
        } else {
            y->nrt = (d->N + 15) / 16;
            y->rows = d->N;
            a_bytes += (size_t)y->nrt * y->nkt * 1024;
            int qs = d->qi + d->qk;
            if (y->has_bias) {
                const int e = bias_qs(d, d->qi, i, &qs);
                if (e) return e;
            }
            y->bias_sh = qs - d->qb;
            y->out_sh = 15 - qs;
        }
        y->bias_sh = clampi(y->bias_sh, -63, 63);
        y->out_sh = clampi(y->out_sh, -63, 62);
        rows_total += 16 * y->nrt;
    }
    g->n_lstm = n_lstm;
    g->nout = L[nl - 1].N;
    /* every layer its own accumulator width (layer_func[i]); acc32 = all
     * layers _acc32b, mixed_acc = both kinds (the fused path only) */
    g->acc32 = 1;
    g->mixed_acc = 0;
    for (int i = 0; i < nl; ++i) {
        g->acc32 &= L[i].acc32 != 0;
        if (L[i].acc32 != L[0].acc32) g->mixed_acc = 1;
    }
    /* NNSPClass_exec copies the last layer into its static int32_t
     * output[50] (nn_speech.c:78, neural_nets.c:152-167): 50 int32 or 100
     * int16; a direct image (one NeuralNetClass_exe / fc_8x16 call) returns
     * the whole activation row */
    if (!direct && g->nout > (L[nl - 1].type == NN_FC && L[nl - 1].act == 3 ? NN_MAX_OUT_LIN : NN_MAX_OUT)) {
        nnsp_set_error("output width %d exceeds NNSPClass_exec's output buffer (50 int32 / 100 int16)", g->nout);
        return NNSP_EUNSUPPORTED;
    }
    im->a_bytes = a_bytes;
    im->rows_total = rows_total;
    im->A = (uint8_t *)calloc(a_bytes ? a_bytes : 1, 1);
    im->wsum = (int32_t *)calloc((size_t)rows_total, sizeof(int32_t));
    im->wsum_r = (int32_t *)calloc((size_t)rows_total, sizeof(int32_t));
    im->bias = (int16_t *)calloc((size_t)rows_total, sizeof(int16_t));
    if (!im->A || !im->wsum || !im->wsum_r || !im->bias) return NNSP_ENOMEM;

    for (int i = 0; i < nl; ++i) {
        const nnsp_layer_desc *d = &L[i];
        const NnLayer *y = &g->L[i];
        const int lstm = d->type == NN_LSTM;
        const int rows_nat = lstm ? 4 * d->N : d->N;
        int8_t *nat = (int8_t *)calloc((size_t)rows_nat * d->K, 1);
        int8_t *natr = lstm ? (int8_t *)calloc((size_t)rows_nat * d->N, 1) : NULL;
        int16_t *bnat = (int16_t *)calloc((size_t)rows_nat, sizeof(int16_t));
        if (!nat || !bnat || (lstm && !natr)) return NNSP_ENOMEM;
        if (lstm) {
            unpack_lstm(d->W, d->N, d->K, nat, d->portable);
            unpack_lstm(d->Wr, d->N, d->N, natr, d->portable);
            if (d->B) unpack_lstm_bias(d->B, d->N, bnat);
            put_frags(im->A + y->a_off, nat, d->K, y->nrt, y->nkt, d->N, 1);
            put_frags(im->A + y->ar_off, natr, d->N, y->nrt, y->nkt_r, d->N, 1);
        } else {
            unpack_fc(d->W, d->N, d->K, nat, d->portable);
            if (d->B) memcpy(bnat, d->B, (size_t)d->N * sizeof(int16_t));
            put_frags(im->A + y->a_off, nat, d->K, y->nrt, y->nkt, d->N, 0);
        }
        for (int p = 0; p < 16 * y->nrt; ++p) {
            const int row = lstm ? lstm_row(p, d->N) : (p < d->N ? p : -1);
            int32_t sw = 0, swr = 0;
            int16_t bv = 0;
            if (row >= 0) {
                for (int k = 0; k < d->K; ++k) sw += nat[(size_t)row * d->K + k];
                if (lstm)
                    for (int k = 0; k < d->N; ++k) swr += natr[(size_t)row * d->N + k];
                bv = bnat[row];
            }
            im->wsum[y->ep_off + p] = 128 * sw;
            im->wsum_r[y->ep_off + p] = 128 * swr;
            im->bias[y->ep_off + p] = bv;
        }
        free(nat);
        free(natr);
        free(bnat);
    }
    return 0;
}

int nnsp_image_upload(nnsp_image *im, void *stream)
{
    int e;
    if ((e = nnspk_malloc(&im->dA, im->a_bytes))) return e;
    if ((e = nnspk_malloc(&im->dwsum, (size_t)im->rows_total * 4))) return e;
    if ((e = nnspk_malloc(&im->dwsum_r, (size_t)im->rows_total * 4))) return e;
    if ((e = nnspk_malloc(&im->dbias, (size_t)im->rows_total * 2))) return e;
    if ((e = nnspk_h2d(im->dA, im->A, im->a_bytes, stream))) return e;
    if ((e = nnspk_h2d(im->dwsum, im->wsum, (size_t)im->rows_total * 4, stream))) return e;
    if ((e = nnspk_h2d(im->dwsum_r, im->wsum_r, (size_t)im->rows_total * 4, stream))) return e;
    if ((e = nnspk_h2d(im->dbias, im->bias, (size_t)im->rows_total * 2, stream))) return e;
    if ((e = nnspk_sync(stream))) return e;
    im->img.A = (const uint8_t *)im->dA;
    im->img.wsum = (const int32_t *)im->dwsum;
    im->img.wsum_r = (const int32_t *)im->dwsum_r;
    im->img.bias = (const int16_t *)im->dbias;
    return 0;
}

void nnsp_image_free(nnsp_image *im)
{
    nnspk_free(im->dA);
    nnspk_free(im->dwsum);
    nnspk_free(im->dwsum_r);
    nnspk_free(im->dbias);
    free(im->A);
    free(im->wsum);
    free(im->wsum_r);
    free(im->bias);
    memset(im, 0, sizeof *im);
}
