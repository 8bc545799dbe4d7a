#!/bin/bash
# round-3 GPU check after the N3 generalisation (fused nn_kernel, wide / multi-LSTM / mixed-acc nets)
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 900 python -u -m pytest tests/test_gpu_refnets.py tests/test_gpu_legacy_portable.py tests/test_gpu_legacy.py tests/test_gpu_nnsp.py tests/test_gpu_nnsp_e2e.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03/t2_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r03/t2_pytest.log; exit 1; }
tail -3 gpurun_out/r03/t2_pytest.log
