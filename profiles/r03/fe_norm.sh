#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_nnsp.py tests/test_gpu_cascade.py tests/test_gpu_configs.py tests/test_gpu_portable.py > gpurun_out/r03/fe_norm_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03/fe_norm_pytest.log; exit 1; }
tail -1 gpurun_out/r03/fe_norm_pytest.log
bash profiles/r03/ab.sh NNSP_LIB "abtest/base/nnsp_amd/libnnsp_mi355x.so -" 4
bash profiles/r03/fe_pmc.sh gpurun_out/r03/pmc_fe_norm | grep -E "fe_kernel|INSTS_VALU|LDS_BANK|GRBM|LDS_IDX|WAIT_ANY"
OUTD=r03/kt2 bash profiles/r03/trace.sh
