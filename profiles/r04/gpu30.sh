#!/bin/bash
# FE addresses: PCM windows through a buffer descriptor on the wave-uniform row (no per-lane 64-bit
# address math), ring stores at a wave-uniform row base; bank sums unconditional (shared mode).
# GPU suite, cascade A/B against HEAD~ (r4f), VAD single-net A/B (batch pair kernel)
set -o pipefail
O=gpurun_out/r04/g30; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest30.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest30.log; exit 1; }
tail -1 $O/pytest30.log
bash profiles/r04/ab.sh NNSP_LIB "abtest/r4f/nnsp_amd/libnnsp_mi355x.so -" 4 || exit 1
bash profiles/r04/ab.sh NNSP_LIB "abtest/r4f/nnsp_amd/libnnsp_mi355x.so -" 3 --net vad || exit 1
echo all-ok
