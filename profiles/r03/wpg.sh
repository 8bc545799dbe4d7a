#!/bin/bash
# fe_kernel with 8 waves per workgroup (one table staging per 8 frames in flight): GPU suite, paired A/B vs 4 waves
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/wpg_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03/wpg_pytest.log; exit 1; }
tail -1 gpurun_out/r03/wpg_pytest.log
bash profiles/r03/ab.sh NNSP_LIB "abtest/w4/libnnsp_mi355x.so -" 4
