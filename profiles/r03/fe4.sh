#!/bin/bash
# fe_kernel4 check: FE parity tests, then paired A/B against the previous FE kernels
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_nnsp.py tests/test_gpu_cascade.py tests/test_gpu_benchcfg.py tests/test_gpu_configs.py > gpurun_out/r03/fe4_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03/fe4_pytest.log; exit 1; }
tail -1 gpurun_out/r03/fe4_pytest.log
bash profiles/r03/ab.sh NNSP_FE4 "0 1" 3
bash profiles/r03/ab.sh NNSP_FE4 "0 1" 2 --net vad
