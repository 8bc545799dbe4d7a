#!/bin/bash
# round-3 GPU check: new config-size / full-scale tests, the nnsp suite, a default bench line
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_nnsp_e2e.py tests/test_gpu_legacy_portable.py tests/test_gpu_nnsp.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03/t1_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03/t1_pytest.log; exit 1; }
tail -3 gpurun_out/r03/t1_pytest.log
timeout -k 10 300 python bench.py > gpurun_out/r03/t1_bench.json 2> gpurun_out/r03/t1_bench.err || { echo "bench failed"; tail -20 gpurun_out/r03/t1_bench.err; exit 1; }
cat gpurun_out/r03/t1_bench.json
