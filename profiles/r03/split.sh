#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03
export NNSP_FE_SPLIT=4
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_cascade.py tests/test_gpu_benchcfg.py tests/test_gpu_configs.py > gpurun_out/r03/split_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03/split_pytest.log; exit 1; }
tail -1 gpurun_out/r03/split_pytest.log
unset NNSP_FE_SPLIT
bash profiles/r03/ab.sh NNSP_FE_SPLIT "1 2 4 8" 3
