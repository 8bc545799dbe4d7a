#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03
export NNSP_FE_PAIR=2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_nnsp.py tests/test_gpu_cascade.py tests/test_gpu_configs.py tests/test_gpu_portable.py tests/test_gpu_benchcfg.py > gpurun_out/r03/fe2_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03/fe2_pytest.log; exit 1; }
tail -1 gpurun_out/r03/fe2_pytest.log
unset NNSP_FE_PAIR
bash profiles/r03/ab.sh NNSP_FE_PAIR "1 2" 4
bash profiles/r03/ab.sh NNSP_LIB "abtest/base/nnsp_amd/libnnsp_mi355x.so -" 3 --net vad
