/*
 * calibrate.c -- CONTAINER-ONLY TEST INFRASTRUCTURE (oracle/tools/calibrate.sh).
 *
 * Times the reference's own NN forward (NeuralNetClass_exe of the portable
 * ARM_OPTIMIZED=0 build, linked here from the reference sources where they
 * lie, on the def_nn*.c nets) against the oracle's restatement
 * (or_net_forward, the shipped semantics) on the same core, both gcc -O3
 * -march=native: the ratio relates the GPU box's oracle CPU baseline to the
 * reference (SURVEY 8(d) "calibration").  The portable build
 * walks the weights in its own byte order, so its outputs on the shipped
 * tables are not meaningful -- only its time is (the MAC count per call is the
 * same).  The front end has no buildable reference here (CMSIS arm_rfft_q31 is
 * binary-only), so only the NN half is calibrated.
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include "neural_nets.h"
#include "../nnsp_oracle.h"

extern NeuralNetClass net_vad, net_kws_galaxy, net_s2i;

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static void to_oracle(const NeuralNetClass *n, or_net *o)
{
    memset(o, 0, sizeof *o);
    o->nl = n->numlayers;
    for (int i = 0; i <= n->numlayers; ++i) o->size[i] = n->size_layer[i];
    for (int i = 0; i < n->numlayers; ++i) {
        o->type[i] = n->net_layer_type[i] == lstm ? OR_LSTM : OR_FC;
        o->qk[i] = n->qbit_kernel[i];
        o->qi[i] = n->qbit_input[i];
        o->qb[i] = n->qbit_bias[i];
        o->act[i] = (int)n->activation_type[i]; /* relu6 0, ftanh 1, fsigmoid 2, linear 3 */
        o->W[i] = n->pt_kernel[i];
        o->Wr[i] = n->pt_kernel_rec[i];
        o->B[i] = n->pt_bias[i];
    }
}

int main(int argc, char **argv)
{
    const int iters = argc > 1 ? atoi(argv[1]) : 20000;
    NeuralNetClass *nets[3] = {&net_vad, &net_kws_galaxy, &net_s2i};
    const char *names[3] = {"vad", "kws", "s2i"};
    int16_t x[240];
    int32_t out[160];
    uint32_t z = 12345;
    printf("{");
    for (int k = 0; k < 3; ++k) {
        NeuralNetClass *n = nets[k];
        or_net on;
        to_oracle(n, &on);
        static or_stream st;
        or_nn_reset(&on, &st);
        NeuralNetClass_setDefault(n);
        double best_r = 1e9, best_o = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
            double t0 = now();
            for (int i = 0; i < iters; ++i) {
                for (int j = 0; j < 240; j += 16) { z = z * 1664525u + 1013904223u; x[j] = (int16_t)(z >> 20) - 2048; }
                NeuralNetClass_exe(n, x, out, -1);
            }
            double t1 = now();
            for (int i = 0; i < iters; ++i) {
                for (int j = 0; j < 240; j += 16) { z = z * 1664525u + 1013904223u; x[j] = (int16_t)(z >> 20) - 2048; }
                or_net_forward(&on, &st, x, out, -1);
            }
            double t2 = now();
            if (t1 - t0 < best_r) best_r = t1 - t0;
            if (t2 - t1 < best_o) best_o = t2 - t1;
        }
        printf("%s\"%s\": {\"reference_us\": %.3f, \"oracle_us\": %.3f, \"reference_over_oracle\": %.3f}", k ? ", " : "",
               names[k], 1e6 * best_r / iters, 1e6 * best_o / iters, best_r / best_o);
    }
    printf("}\n");
    return 0;
}
