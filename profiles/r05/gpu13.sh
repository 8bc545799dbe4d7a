#!/bin/bash
# early return (NNSP_EARLY_RETURN=1: the call returns once the rounds are done; the next round 0 waits for the
# look-ahead front end on the device): cascade suites with it on, A/B; then plain vs torchrun at world size 1
set -o pipefail
O=gpurun_out/r05/g13; mkdir -p $O
export TMPDIR=/tmp
NNSP_EARLY_RETURN=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cascade.py tests/test_gpu_benchloop.py tests/test_gpu_cascade_state.py tests/test_gpu_benchcfg.py tests/test_gpu_shards.py > $O/pytest_early.log 2>&1 || { echo "early pytest failed"; tail -40 $O/pytest_early.log; exit 1; }
tail -1 $O/pytest_early.log
bash profiles/r05/ab.sh NNSP_EARLY_RETURN "- 1" 3 || exit 1
bash profiles/r05/gpu12.sh || exit 1
echo all-ok
