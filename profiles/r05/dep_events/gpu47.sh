#!/bin/bash
# stream-ordering events without timestamps (NNSP_DEP_EVENTS=1): cascade suites with it on, then paired A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/depev
mkdir -p $O
timeout -k 10 600 env NNSP_DEP_EVENTS=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_cascade.py tests/test_gpu_benchloop.py tests/test_gpu_cascade_state.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash profiles/r05/ab2.sh depev "- NNSP_DEP_EVENTS=1" 5 || exit 1
echo all-ok
