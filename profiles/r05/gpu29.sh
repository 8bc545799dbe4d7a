#!/bin/bash
# the chunk's tail copy / counter clear after VAD's round 0 (NNSP_BEHIND=1); round-0 cold front end grid 256
set -o pipefail
O=gpurun_out/r05/g29; mkdir -p $O
export TMPDIR=/tmp
NNSP_BEHIND=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cascade.py tests/test_gpu_benchloop.py tests/test_gpu_cascade_state.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash profiles/r05/ab2.sh behind "- NNSP_BEHIND=1 NNSP_COLD_FE_BLOCKS=256" 5 || exit 1
echo all-ok
