#!/bin/bash
# prebuilt front-end tables: full GPU suite, paired A/B against the previous build (NNSP_LIB), per-wave FE staging probe
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/fetab_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03/fetab_pytest.log; exit 1; }
tail -1 gpurun_out/r03/fetab_pytest.log
bash profiles/r03/ab.sh NNSP_LIB "abtest/base/nnsp_amd/libnnsp_mi355x.so -" 3 && bash profiles/r03/ab.sh NNSP_LIB "abtest/base/nnsp_amd/libnnsp_mi355x.so -" 2 --net vad || exit 1
timeout -k 10 120 python profiles/r02/proj_waves.py vad 26624 2>&1 | grep -v amdgpu.ids
VAR=NNSP_NONE VALS="-" bash profiles/r03/cofe_trace.sh && python3 profiles/r03/chunk_timeline.py $(find gpurun_out/r03/ct_- -name "*kernel_trace.csv" | head -1) 3 > gpurun_out/r03/ct_-/timeline3.txt
