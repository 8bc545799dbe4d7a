#!/bin/bash
# look-ahead front end after the third-last round's proj when the last chunk needed many rounds (NNSP_AHEAD_LATE=1)
set -o pipefail
O=gpurun_out/r05/g36; mkdir -p $O
export TMPDIR=/tmp
NNSP_AHEAD_LATE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cascade.py tests/test_gpu_benchloop.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash profiles/r05/ab2.sh aheadlate "- NNSP_AHEAD_LATE=1" 4 || exit 1
echo all-ok
