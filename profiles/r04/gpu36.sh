#!/bin/bash
# round-0 launch order: 1 (default: VAD, S2I, KWS), 4 (KWS, S2I, VAD), 5 (VAD, KWS, S2I); nothing waits
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_cascade.py > gpurun_out/pytest36.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/pytest36.log; exit 1; }
tail -1 gpurun_out/pytest36.log
NNSP_R0_ORDER=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_cascade.py > gpurun_out/pytest36_4.log 2>&1 || { echo "pytest order 4 failed"; tail -20 gpurun_out/pytest36_4.log; exit 1; }
tail -1 gpurun_out/pytest36_4.log
bash profiles/r04/ab.sh NNSP_R0_ORDER "- 4 5" 3 || exit 1
echo all-ok
