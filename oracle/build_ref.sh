#!/usr/bin/env bash
# Container-only: compile reference ns-nnsp C files, where they lie under
# /root/reference, with the host gcc -- no stand-in headers, no stand-in
# libraries, no copied sources.  Outputs go to oracle/_ref/ only (git-ignored).
# TEST INFRASTRUCTURE ONLY: the checker of the oracle, never the product.
#
#  libnnsp_ref_partial.so      the shipped (ARM_OPTIMIZED=1) build's files that
#                              compile as they are: activation, fixlog10, mel,
#                              window, spectrogram_module, feature_module,
#                              neural_nets, nn_speech, lstm.  Left out:
#                              affine.c / affine_acc32b.c (their ARM path needs
#                              the ARM DSP intrinsics, which the vendored
#                              cmsis_gcc.h defines only as ARM asm) and
#                              fft_arm.c (calls CMSIS-DSP arm_rfft_q31, shipped
#                              only as a Cortex-M binary).  Their symbols stay
#                              undefined (loaded with RTLD_LAZY; never reached).
#  libnnsp_ref_nn_portable.so  the reference's own portable NN build: affine.c,
#                              affine_acc32b.c, lstm.c, neural_nets.c,
#                              activation.c with the reference's compile-time
#                              switches set on the command line
#                              (ambiq_nnsp_debug.h's guard macro predefined,
#                              AMBIQ_NNSP_DEBUG=0, ARM_OPTIMIZED=0) and the
#                              vendored CMSIS Core include for cmsis_gcc.h.
#                              Same arithmetic as the shipped path after the MAC
#                              loop (affine.c:186-253 vs :311-339); it walks the
#                              weights in the portable order and applies the
#                              align shift that is dead in the shipped build (T1).
#  libnnsp_ref_fe_portable.so  the reference's portable front end
#                              (ARM_OPTIMIZED=0: fft.c, complex.c,
#                              twiddle_fft_dif.c, spectrogram_module.c,
#                              feature_module.c, mel, log10, window), row N4.
#  libnnsp_ref_nnsp_portable.so  the whole portable path: nn_speech.c
#                              (NNSPClass_init/_reset/_exec) over the portable
#                              front end and NN files above, same switches.
#  libnnsp_ref_nets.so         evb/src/def_nn{0_s2i,1_vad,2_kws_galaxy}.c (the
#                              reference's three nets as data) against the
#                              reference headers, linked with the portable NN
#                              build so their layer_func addresses resolve.
set -euo pipefail
REF=${REF:-/root/reference}
OUT=$(cd "$(dirname "$0")" && pwd)/_ref
[ -d "$REF/ns-nnsp/src" ] || { echo "reference not present: skip"; exit 0; }
mkdir -p "$OUT"
SRC=$REF/ns-nnsp/src
API=$REF/ns-nnsp/includes-api
CORE=$REF/evb/includes/extern/CMSIS/CMSIS_5-5.9.0/CMSIS/Core/Include

gcc -O2 -fPIC -shared -w -fwrapv -I"$API" \
    "$SRC/activation.c" "$SRC/fixlog10.c" "$SRC/melSpecProc.c" "$SRC/melSpec_coeff.c" \
    "$SRC/window_stft_coef.c" "$SRC/spectrogram_module.c" "$SRC/feature_module.c" \
    "$SRC/neural_nets.c" "$SRC/nn_speech.c" "$SRC/lstm.c" \
    -o "$OUT/libnnsp_ref_partial.so"

gcc -O2 -fPIC -shared -w -fwrapv -D__AMBIQ_NNSP_DEBUG__ -DAMBIQ_NNSP_DEBUG=0 -DARM_OPTIMIZED=0 \
    -I"$API" -I"$CORE" \
    "$SRC/affine.c" "$SRC/affine_acc32b.c" "$SRC/lstm.c" "$SRC/neural_nets.c" "$SRC/activation.c" \
    -Wl,-z,defs -o "$OUT/libnnsp_ref_nn_portable.so"

gcc -O2 -fPIC -shared -w -I"$API" \
    "$REF/evb/src/def_nn0_s2i.c" "$REF/evb/src/def_nn1_vad.c" "$REF/evb/src/def_nn2_kws_galaxy.c" \
    -L"$OUT" -lnnsp_ref_nn_portable -Wl,-rpath,'$ORIGIN' -Wl,-z,defs -o "$OUT/libnnsp_ref_nets.so"

# the reference's own portable front end (ARM_OPTIMIZED=0, row N4): fft.c's
# radix-4 DIF FFT and rfft split, complex.c, twiddle_fft_dif.c, and the
# FeatureClass / stftModule / Mel / log10 files built with the same switches
gcc -O2 -fPIC -shared -w -fwrapv -D__AMBIQ_NNSP_DEBUG__ -DAMBIQ_NNSP_DEBUG=0 -DARM_OPTIMIZED=0 \
    -I"$API" -I"$CORE" \
    "$SRC/fft.c" "$SRC/complex.c" "$SRC/twiddle_fft_dif.c" "$SRC/spectrogram_module.c" "$SRC/feature_module.c" \
    "$SRC/melSpecProc.c" "$SRC/melSpec_coeff.c" "$SRC/fixlog10.c" "$SRC/window_stft_coef.c" \
    -Wl,-z,defs -o "$OUT/libnnsp_ref_fe_portable.so"

# the reference timed beside the oracle on the same cores (container
# calibration, BASELINE.md / SURVEY 8(d)): -O3 -march=native like the oracle
gcc -O3 -march=native -fPIC -shared -w -fwrapv -D__AMBIQ_NNSP_DEBUG__ -DAMBIQ_NNSP_DEBUG=0 -DARM_OPTIMIZED=0 \
    -I"$API" -I"$CORE" \
    "$SRC/affine.c" "$SRC/affine_acc32b.c" "$SRC/lstm.c" "$SRC/neural_nets.c" "$SRC/activation.c" \
    -Wl,-z,defs -o "$OUT/libnnsp_ref_nn_portable_o3.so"

# the reference's whole portable NNSP path (ARM_OPTIMIZED=0): NNSPClass_init /
# _reset / _exec of nn_speech.c over the portable front end and NN, for the
# end-to-end fixture ref_nnsp_portable.npz
gcc -O2 -fPIC -shared -w -fwrapv -D__AMBIQ_NNSP_DEBUG__ -DAMBIQ_NNSP_DEBUG=0 -DARM_OPTIMIZED=0 \
    -I"$API" -I"$CORE" \
    "$SRC/nn_speech.c" "$SRC/feature_module.c" "$SRC/spectrogram_module.c" "$SRC/fft.c" "$SRC/complex.c" \
    "$SRC/twiddle_fft_dif.c" "$SRC/melSpecProc.c" "$SRC/melSpec_coeff.c" "$SRC/fixlog10.c" \
    "$SRC/window_stft_coef.c" "$SRC/affine.c" "$SRC/affine_acc32b.c" "$SRC/lstm.c" "$SRC/neural_nets.c" \
    "$SRC/activation.c" -Wl,-z,defs -o "$OUT/libnnsp_ref_nnsp_portable.so"
echo "$OUT"
