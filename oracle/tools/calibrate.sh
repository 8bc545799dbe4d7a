#!/usr/bin/env bash
# CONTAINER-ONLY: build oracle/tools/calibrate.c against the reference's own
# NN sources and def_nn*.c (compiled where they lie, ARM_OPTIMIZED=0, no
# stand-ins) and the oracle, all -O3 -march=native, into oracle/_ref/, and run
# it.  Output: JSON, per net, microseconds per NeuralNetClass_exe.
set -euo pipefail
REF=${REF:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=$HERE/../_ref
[ -d "$REF/ns-nnsp/src" ] || { echo "reference not present: skip"; exit 0; }
mkdir -p "$OUT"
SRC=$REF/ns-nnsp/src
gcc -O3 -march=native -w -fwrapv -D__AMBIQ_NNSP_DEBUG__ -DAMBIQ_NNSP_DEBUG=0 -DARM_OPTIMIZED=0 \
    -I"$REF/ns-nnsp/includes-api" -I"$REF/evb/includes/extern/CMSIS/CMSIS_5-5.9.0/CMSIS/Core/Include" \
    "$HERE/calibrate.c" "$HERE/../nnsp_oracle.c" \
    "$SRC/affine.c" "$SRC/affine_acc32b.c" "$SRC/lstm.c" "$SRC/neural_nets.c" "$SRC/activation.c" \
    "$REF/evb/src/def_nn0_s2i.c" "$REF/evb/src/def_nn1_vad.c" "$REF/evb/src/def_nn2_kws_galaxy.c" \
    -o "$OUT/calibrate"
"$OUT/calibrate" "${1:-20000}"
