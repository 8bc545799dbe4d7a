#!/bin/bash
# the early-return book stream created only when used (a fifth HIP stream otherwise) vs always (abtest/prev)
set -o pipefail
O=gpurun_out/r05/g23; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cascade.py tests/test_gpu_cascade_state.py tests/test_gpu_benchloop.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash profiles/r05/ab2.sh bstream "NNSP_LIB=abtest/prev/nnsp_amd/libnnsp_mi355x.so -" 5 || exit 1
echo all-ok
