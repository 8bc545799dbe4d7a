#!/bin/bash
# FE: first window issued before table staging -- cascade + FE parity, paired A/B vs the previous build, staging probe
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest tests/test_gpu_cascade.py tests/test_gpu_benchcfg.py tests/test_gpu_configs.py tests/test_gpu_nnsp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/early_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03/early_pytest.log; exit 1; }
tail -1 gpurun_out/r03/early_pytest.log
bash profiles/r03/ab.sh NNSP_LIB "abtest/base/nnsp_amd/libnnsp_mi355x.so -" 4 || exit 1
timeout -k 10 300 python -u profiles/r03/wg_timeline.py 32768 gpurun_out/r03/wg_records2.npz > gpurun_out/r03/wg_timeline2.txt 2>&1 || { tail -5 gpurun_out/r03/wg_timeline2.txt; exit 1; }
python3 -c "
import numpy as np
d=np.load('gpurun_out/r03/wg_records2.npz'); a=d['fe']
print('fe staging med', np.median((a[:,1]-a[:,0])/100.0), 'us; life med', np.median((a[:,2]-a[:,0])/100.0))"
