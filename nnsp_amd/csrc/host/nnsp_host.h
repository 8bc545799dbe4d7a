/* nnsp_host.h -- internal declarations of the C host library. */
#ifndef NNSP_HOST_H
#define NNSP_HOST_H
#include <stddef.h>
#include <stdint.h>

#include "../../../include/nnsp_api.h"
#include "../kernels/nnsp_kabi.h"

/* error codes (negative: argument/validation; positive: HIP runtime) */
#define NNSP_EINVAL (-1)
#define NNSP_EUNSUPPORTED (-2)
#define NNSP_ENOMEM (-3)

/* One layer as the engine sees it (what a NeuralNetClass row describes). */
typedef struct {
    int type;                 /* NN_FC / NN_LSTM */
    int K, N;                 /* input width, output width (LSTM: units) */
    int act;                  /* device activation enum (FC only) */
    int acc32;
    int qk, qb, qi, qir;
    const int8_t *W, *Wr;     /* interleaved byte streams (def_nn*.c layout) */
    const int16_t *B;         /* NULL: no bias */
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
                     int thresh_prob, int th_count);
int nnsp_image_upload(nnsp_image *im, void *stream);
void nnsp_image_free(nnsp_image *im);

/* activation function pointer -> device enum (-1 unknown) */
int nnsp_act_of(void *(*fn)(void *, int32_t *, int));

void nnsp_set_error(const char *fmt, ...);
const char *nnsp_last_error(void);

#endif
