#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_nnsp.py tests/test_gpu_cascade.py tests/test_gpu_benchcfg.py tests/test_gpu_configs.py tests/test_gpu_refnets.py > gpurun_out/r03/proj1_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03/proj1_pytest.log; exit 1; }
tail -1 gpurun_out/r03/proj1_pytest.log
bash profiles/r03/nn_pmc.sh gpurun_out/r03/pmc_proj_vad proj_kernel --net vad
for n in vad cascade; do timeout -k 10 200 python bench.py --no-cpu-baseline --no-stress --net $n > gpurun_out/r03/proj1_$n.json 2>/dev/null && python -c "import json; d=json.load(open('gpurun_out/r03/proj1_$n.json')); print('$n', d['value']/1e6, d['ms_per_step'], d.get('nn_ms_per_step'))"; done
