#!/bin/bash
# S2I's post-processing on a 13th wave (PIPE_S2I_SPLIT=1 library) with round 0 launching S2I first
set -o pipefail
O=gpurun_out/r05/g28; mkdir -p $O
export TMPDIR=/tmp
NNSP_LIB=abtest/split/nnsp_amd/libnnsp_mi355x.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cascade.py tests/test_gpu_benchcfg.py tests/test_gpu_refnets.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash profiles/r05/ab2.sh s2isplit "- NNSP_LIB=abtest/split/nnsp_amd/libnnsp_mi355x.so" 5 || exit 1
echo all-ok
