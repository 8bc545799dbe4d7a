/*
 * nnsp_api.h -- drop-in declarations of the ns-nnsp C API, served by
 * libnnsp_mi355x.so (MI355X / gfx950 implementation).
 *
 * One header declares the whole legacy surface.  The reference spreads the
 * same declarations over ns-nnsp/includes-api/ (19 headers); thin forwarding headers
 * with those file names live next to this one so that unchanged net
 * definition files (evb/src/def_nn*.c, which include "neural_nets.h",
 * "activation.h", "affine.h", "affine_acc32b.h", "lstm.h") compile against
 * this library.
 *
 * Struct layouts, enum values and prototypes are ABI-identical to the
 * reference (same member order and types; compile the def files with the same
 * host compiler as this library).  Citations are to /root/reference.
 */
#ifndef NNSP_API_H
#define NNSP_API_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- constants: ambiq_nnsp_const.h:3-10, ambiq_stdint.h:3-7,
 *      nnsp_identification.h:3-9, s2i_const.h:3-4, ambiq_nnsp_debug.h:3-4 ---- */
#define LEN_FFT_NNSP 512
#define LEN_STFT_WIN_COEFF 480
#define LEN_STFT_HOP 160
#define NUM_MELBANKS 40
#define NUM_FEATURE_CONTEXT 6
#define MAX_SIZE_FEATURE 50
#define DIMEMSION_FEATURE NUM_MELBANKS
#define SAMPLING_RATE 16000

#define MAX_INT32_T ((int32_t)0x7fffffff)
#define MIN_INT32_T ((int32_t)0x80000000)
#define MAX_INT16_T ((int16_t)0x7fff)
#define MIN_INT16_T ((int16_t)0x8000)
#define ONE_N32_Q15 ((int32_t)32768)

#define DIM_INTENTS 7
#define DIM_SLOTS 17

#define AMBIQ_NNSP_DEBUG 0
#ifndef ARM_OPTIMIZED
#define ARM_OPTIMIZED 1 /* the shipped build: CMSIS q31 rFFT + interleaved weights */
#endif

#ifndef MAX
#define MAX(x, y) (((x) > (y)) ? (x) : (y))
#endif
#ifndef MIN
#define MIN(x, y) (((x) < (y)) ? (x) : (y))
#endif

typedef enum { s2i_id = 0, vad_id = 1, kws_galaxy_id = 2, num_NNSP_IDS = 3 } NNSP_ID;

/* ---- activations: activation.h:8-22 ---- */
typedef enum { relu6, ftanh, sigmoid, linear } ACTIVATION_TYPE;

void *relu6_fix(int16_t *y, int32_t *x, int len);   /* Q15 in -> Q12 out */
void *linear_fix(int32_t *y, int32_t *x, int len);  /* Q15 copy (int32)   */
void *tanh_fix(int16_t *y, int32_t *x, int len);
void *sigmoid_fix(int16_t *y, int32_t *x, int len);

/* ---- 8x16 affine / recurrent kernels: affine.h:19-82, affine_acc32b.h:26-89 ---- */
typedef void *(*nnsp_act_fn)(void *, int32_t *, int);

int affine_Krows_8x16(int16_t dim_output, int16_t **pp_output, int8_t **pp_kernel,
                      int16_t **pp_bias, int16_t *input, int16_t dim_input,
                      int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input,
                      int64_t *pt_accum, int8_t is_out, void *(*act)(void *, int32_t *, int));
int affine_Krows_8x16_acc32b(int16_t dim_output, int16_t **pp_output, int8_t **pp_kernel,
                             int16_t **pp_bias, int16_t *input, int16_t dim_input,
                             int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input,
                             int32_t *pt_accum, int8_t is_out,
                             void *(*act)(void *, int32_t *, int));

int rc_Krows_8x16(int16_t dim_output, int16_t **pp_output, int8_t **pp_kernel,
                  int8_t **pp_kernel_rec, int16_t **pp_bias, int16_t *input, int16_t *input_rec,
                  int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel,
                  int16_t qbit_bias, int16_t qbit_input, int16_t qbit_input_rec,
                  void *(*act)(void *, int32_t *, int));
int rc_Krows_8x16_acc32b(int16_t dim_output, int16_t **pp_output, int8_t **pp_kernel,
                         int8_t **pp_kernel_rec, int16_t **pp_bias, int16_t *input,
                         int16_t *input_rec, int16_t dim_input, int16_t dim_input_rec,
                         int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input,
                         int16_t qbit_input_rec, void *(*act)(void *, int32_t *, int));

/* Layer entry points; NeuralNetClass.layer_func[] holds their addresses. */
int fc_8x16(int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias,
            int16_t *input, int16_t *input_rec, int32_t *c_state, int16_t dim_output,
            int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel, int16_t qbit_bias,
            int16_t qbit_input, int16_t qbit_input_rec, ACTIVATION_TYPE act_type,
            void *(*act)(void *, int32_t *, int));
int fc_8x16_acc32b(int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias,
                   int16_t *input, int16_t *input_rec, int32_t *c_state, int16_t dim_output,
                   int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel,
                   int16_t qbit_bias, int16_t qbit_input, int16_t qbit_input_rec,
                   ACTIVATION_TYPE act_type, void *(*act)(void *, int32_t *, int));
int rc_8x16(int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias,
            int16_t *input, int16_t *input_rec, int16_t dim_output, int16_t dim_input,
            int16_t dim_input_rec, int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input,
            int16_t qbit_input_rec, ACTIVATION_TYPE act_type,
            void *(*act)(void *, int32_t *, int));
int rc_8x16_acc32b(int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias,
                   int16_t *input, int16_t *input_rec, int16_t dim_output, int16_t dim_input,
                   int16_t dim_input_rec, int16_t qbit_kernel, int16_t qbit_bias,
                   int16_t qbit_input, int16_t qbit_input_rec, ACTIVATION_TYPE act_type,
                   void *(*act)(void *, int32_t *, int));
/* lstm.h:15-49 */
int lstm_8x16(int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec, int16_t *p_bias,
              int16_t *input, int16_t *h_state, int32_t *c_state, int16_t dim_output,
              int16_t dim_input, int16_t dim_input_rec, int16_t qbit_kernel, int16_t qbit_bias,
              int16_t qbit_input, int16_t qbit_input_rec, ACTIVATION_TYPE act_type,
              void *(*act)(void *, int32_t *, int));
int lstm_8x16_acc32b(int16_t *p_output, int8_t *p_kernel, int8_t *p_kernel_rec,
                     int16_t *p_bias, int16_t *input, int16_t *h_state, int32_t *c_state,
                     int16_t dim_output, int16_t dim_input, int16_t dim_input_rec,
                     int16_t qbit_kernel, int16_t qbit_bias, int16_t qbit_input,
                     int16_t qbit_input_rec, ACTIVATION_TYPE act_type,
                     void *(*act)(void *, int32_t *, int));

void shift_64b(int64_t *x, int8_t shift, int len);
void shift_32b(int32_t *x, int8_t shift, int len);

/* ---- NeuralNetClass: neural_nets.h:9-42 ---- */
typedef enum { fc, lstm } NET_LAYER_TYPE;

typedef struct {
    int8_t numlayers;
    int16_t size_layer[11];
    NET_LAYER_TYPE net_layer_type[10];
    int8_t qbit_kernel[10];
    int8_t qbit_input[10];
    int8_t qbit_bias[10];
    ACTIVATION_TYPE activation_type[10];
    int32_t *pt_cstate[10];
    int16_t *pt_hstate[10];
    void *(*act_func[10])(void *, int32_t *, int);
    int *(*layer_func[10])();
    int8_t *pt_kernel[10];
    int16_t *pt_bias[10];
    int8_t *pt_kernel_rec[10];
} NeuralNetClass;

void NeuralNetClass_init(NeuralNetClass *pt_inst);
void NeuralNetClass_setDefault(NeuralNetClass *pt_inst);
void NeuralNetClass_exe(NeuralNetClass *pt_inst, int16_t *input, int32_t *output,
                        int8_t debug_layer);

/* ---- front end: spectrogram_module.h:9-42, feature_module.h:7-28 ---- */
typedef struct {
    int16_t len_win;
    int16_t hop;
    int16_t len_fft;
    int16_t dataBuffer[512];
    const int16_t *window;
} stftModule;

int stftModule_construct(stftModule *ps);
int stftModule_setDefault(stftModule *ps);
void spec2pspec_arm(int32_t *y, int32_t *x, int len);
int stftModule_analyze_arm(void *ps, int16_t *x, int32_t *y);
/* the ARM_OPTIMIZED=0 build's stages (spectrogram_module.c:33-77, fft.h:4-5);
 * exported beside the shipped ones.  rfft: num_rfft 256 or 512 (y: num_rfft/2
 * + 1 complex); fft: exp_nfft 0..8 (in place on its input, like fft.c) -- the
 * sizes fft.c's twiddle and bit-reversal tables serve; others return with
 * nnsp_legacy_status() = NNSP_EUNSUPPORTED */
void spec2pspec(int32_t *y, int32_t *x, int len);
int stftModule_analyze(stftModule *ps, int16_t *x, int32_t *y);
void rfft(int num_rfft, int32_t *input, void *output_);
void fft(int exp_nfft, void *input_, void *output_);

/* complex.h (the ARM_OPTIMIZED=0 build's complex helpers, complex.c):
 * int64 products with int32 clamps where complex.c has them, int32 wrap
 * elsewhere.  complex32_sub negates *b in place, as complex.c:108-113 does. */
typedef struct {
    int32_t real;
    int32_t imag;
} COMPLEX32;
typedef struct {
    int16_t real;
    int16_t imag;
} COMPLEX16;
void complex32_copy(COMPLEX32 *dst, COMPLEX32 *src);
void complex32_affine(COMPLEX32 *out, COMPLEX32 *Mat, COMPLEX32 *input, int shift_r, int len);
void complex32_interprod(COMPLEX32 *out, COMPLEX32 *arry1, COMPLEX32 *arry2, int shift_r, int len);
void complex32_complex16_elmtprod(COMPLEX32 *out, COMPLEX32 *arry1, COMPLEX16 *arry2, int len);
void complex32_add(COMPLEX32 *out, COMPLEX32 *addr1, COMPLEX32 *addr2);
void complexArry32_add(COMPLEX32 *out, COMPLEX32 *addr1, COMPLEX32 *addr2, int len);
void complex32_neg(COMPLEX32 *out, COMPLEX32 *in);
void complex32_sub(COMPLEX32 *out, COMPLEX32 *a, COMPLEX32 *b);
void complex32_mul(COMPLEX32 *out, COMPLEX32 *addr1, COMPLEX32 *addr2);
void complex32_init(COMPLEX32 *inst, int32_t real, int32_t imag);
void complex32_real2cmplx(COMPLEX32 *inst, int32_t real);
void complexArry32_real2cmplx(COMPLEX32 *inst, int32_t *real, int32_t len);
void complexArry32_init(COMPLEX32 *inst, int32_t *real, int32_t *imag, int len);
void complexArry32_print(COMPLEX32 *inst, int len);

typedef struct {
    stftModule state_stftModule;
    int32_t feature[MAX_SIZE_FEATURE];
    int16_t normFeatContext[NUM_FEATURE_CONTEXT * MAX_SIZE_FEATURE];
    int16_t num_context;
    int16_t dim_feat;
    const int32_t *pt_norm_mean;
    const int32_t *pt_norm_stdR;
    int8_t qbit_output;
} FeatureClass;

void FeatureClass_construct(FeatureClass *ps, const int32_t *norm_mean,
                            const int32_t *norm_stdR, int8_t qbit_output);
void FeatureClass_setDefault(FeatureClass *ps);
void FeatureClass_execute(FeatureClass *ps, int16_t *input);

/* melSpecProc.h:4, fixlog10.h:8-17, fft_arm.h:8-10 */
void melSpecProc(int32_t *specs, int32_t *melSpecs);
void norm_oneTwo(int32_t x, int32_t *y, int8_t *shift);
void my_log10(int32_t *out, int32_t x);
void log10_vec(int32_t *out, int32_t *x, int32_t len, int16_t bit_frac_in);
void arm_fft_init(void);
void arm_fft_exec(int32_t *y /* Q21, 1024 words */, int32_t *x /* Q30, 512(+2) words */);

/* tables exported by the reference library (window_stft_coef.c:3-6,
 * melSpec_coeff.c:3-5, fixlog10.c:6, activation.c:5) */
extern const int16_t len_stft_win_coeff;
extern const int16_t hop;
extern const int16_t stft_win_coeff[];
extern const int16_t num_mfltrBank;
extern const int16_t mfltrBank_coeff[];
extern const int16_t log_tayler_coeff[];
extern int16_t coeffs_tanh[];

/* ---- NNSPClass: nn_speech.h:12-57 ---- */
typedef struct {
    char nn_id;
    void *pt_net;
    void *pt_feat;
    int8_t slides;
    int16_t trigger;
    int16_t *pt_thresh_prob;
    int16_t counts_category[8];
    int16_t *pt_th_count_trigger;
    int16_t num_dnsmpl;
    int16_t outputs[3];
    int16_t argmax_last;
} NNSPClass;

int NNSPClass_init(NNSPClass *pt_inst, void *pt_net, void *pt_feat, char nn_id,
                   const int32_t *pt_mean, const int32_t *pt_stdR, int16_t *pt_thresh_prob,
                   int16_t *pt_th_count_trigger);
int NNSPClass_reset(NNSPClass *pt_inst);
int16_t NNSPClass_exec(NNSPClass *pt_inst, int16_t *rawPCM);
void my_argmax(int32_t *vec, int len, int16_t *Imax);
int32_t compute_pwr2(int32_t input);
int32_t ceiling(int32_t input);
void binary_post_proc(NNSPClass *pt_inst, int32_t *pt_nn_est, int16_t *pt_trigger);
void s2i_post_proc(NNSPClass *pt_inst, int32_t *pt_nn_est, int16_t *pt_trigger);

/* Error channel of this library's single-stream API (not in the reference,
 * whose functions return 0 or void).  A HIP or allocation failure inside any
 * call above makes that call return without touching its outputs (int
 * results: the error code, pointer results: NULL) and records the first such
 * error: nnsp_legacy_status() returns it (0: none; nnsp_strerror() describes
 * it) until nnsp_legacy_clear().  The process is never aborted. */
int nnsp_legacy_status(void);
/* Which build of the reference the drop-in API reproduces (row N4): 1 (the
 * default) the shipped ARM_OPTIMIZED=1 build, 0 the ARM_OPTIMIZED=0 one --
 * FeatureClass_execute / NNSPClass_exec run the portable front end, and
 * NeuralNetClass_exe, fc_8x16, lstm_8x16, affine_Krows_8x16, rc_* read the
 * portable weight order with the live align shift.  The reference fixes this
 * at compile time; here a portable application calls
 * nnsp_set_arm_optimized(0) once, or runs with NNSP_ARM_OPTIMIZED=0 in the
 * environment.  Returns 0, or NNSP_EINVAL (-1) for a value other than 0 / 1. */
int nnsp_set_arm_optimized(int arm_optimized);
int nnsp_get_arm_optimized(void);
void nnsp_legacy_clear(void);

#ifdef __cplusplus
}
#endif
#endif /* NNSP_API_H */
