#!/usr/bin/env bash
# Container-only: compile the reference ns-nnsp C files that build from their
# own sources with the host gcc (no stand-in headers, no stand-in libraries)
# into oracle/_ref/libnnsp_ref_partial.so.  TEST INFRASTRUCTURE ONLY.
#
# Left out, because they cannot be built here without stand-ins:
#   affine.c / affine_acc32b.c  ARM_OPTIMIZED=1 path needs the ARM DSP
#                               intrinsics (__SXTB16/__SMLALD/__SMLAD), which the
#                               vendored cmsis_gcc.h defines only as ARM asm;
#   fft_arm.c                   calls CMSIS-DSP arm_rfft_q31 (ships as a Cortex-M
#                               binary only, evb/libs/libCMSISDSP.a).
# Their symbols stay undefined in the .so (it is loaded with RTLD_LAZY and the
# tests never call a path that reaches them).
set -euo pipefail
REF=${REF:-/root/reference}
OUT=$(cd "$(dirname "$0")" && pwd)/_ref
[ -d "$REF/ns-nnsp/src" ] || { echo "reference not present: skip"; exit 0; }
mkdir -p "$OUT"
SRC=$REF/ns-nnsp/src
gcc -O2 -fPIC -shared -w -fwrapv -I"$REF/ns-nnsp/includes-api" \
    "$SRC/activation.c" "$SRC/fixlog10.c" "$SRC/melSpecProc.c" "$SRC/melSpec_coeff.c" \
    "$SRC/window_stft_coef.c" "$SRC/spectrogram_module.c" "$SRC/feature_module.c" \
    "$SRC/neural_nets.c" "$SRC/nn_speech.c" "$SRC/lstm.c" \
    -o "$OUT/libnnsp_ref_partial.so"
echo "$OUT/libnnsp_ref_partial.so"
