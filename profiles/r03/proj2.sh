#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_nnsp.py tests/test_gpu_cascade.py tests/test_gpu_benchcfg.py tests/test_gpu_configs.py tests/test_gpu_refnets.py tests/test_gpu_nnsp_e2e.py > gpurun_out/r03/proj2_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03/proj2_pytest.log; exit 1; }
tail -1 gpurun_out/r03/proj2_pytest.log
bash profiles/r03/nn_pmc.sh gpurun_out/r03/pmc_proj_vad2 proj_kernel --net vad | grep -E "proj|INSTS_VALU|INSTS_SALU|GRBM|WAVES "
bash profiles/r03/ab.sh NNSP_LIB "abtest/base/nnsp_amd/libnnsp_mi355x.so -" 3 --net vad
bash profiles/r03/ab.sh NNSP_LIB "abtest/base/nnsp_amd/libnnsp_mi355x.so -" 3
