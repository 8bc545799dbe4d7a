#!/bin/bash
# recur_pipe_kernel with per-wave progress flags instead of the per-iteration barrier: GPU suite, per-stage clocks,
# paired A/B against the barrier build (NNSP_LIB)
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/flags_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03/flags_pytest.log; exit 1; }
tail -1 gpurun_out/r03/flags_pytest.log
for n in vad kws s2i; do timeout -k 10 120 python profiles/recur_clocks.py $n 8192 ref 2>&1 | grep -E 'iteration' || exit 1; done
bash profiles/r03/ab.sh NNSP_LIB "abtest/base/nnsp_amd/libnnsp_mi355x.so -" 4 && bash profiles/r03/ab.sh NNSP_LIB "abtest/base/nnsp_amd/libnnsp_mi355x.so -" 2 --net s2i && bash profiles/r03/ab.sh NNSP_LIB "abtest/base/nnsp_amd/libnnsp_mi355x.so -" 2 --net kws
