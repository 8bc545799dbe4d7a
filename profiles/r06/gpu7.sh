#!/bin/bash
# round 6: fused VAD prefix, register-staged sliding window -- parity (required), clocks, paired A/B
set -o pipefail
O=gpurun_out/r06/${TAG:-g7}; mkdir -p $O
export TMPDIR=/tmp
NNSP_FUSE_PREFIX=2 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_benchloop.py tests/test_gpu_benchcfg.py tests/test_gpu_cascade_ref.py > $O/pytest_req.log 2>&1 || { echo "pytest (required) failed"; tail -40 $O/pytest_req.log; exit 1; }
tail -1 $O/pytest_req.log
NNSP_LIB=abtest/p6/nnsp_amd/libnnsp_mi355x.so NNSP_FUSE_PREFIX=1 timeout -k 10 200 python profiles/r06/casc_clocks_fp.py > $O/clk_1.txt 2>&1 || { echo "clocks failed"; tail -20 $O/clk_1.txt; exit 1; }
cat $O/clk_1.txt
bash profiles/r06/ab.sh NNSP_FUSE_PREFIX "0 1" 3 || exit 1
echo all-ok
