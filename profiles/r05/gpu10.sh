#!/bin/bash
# proj padding rows branch-free (default build); S2I with its post-processing on a 13th wave (abtest/split,
# PIPE_S2I_SPLIT=1): suites, A/B against the round start
set -o pipefail
O=gpurun_out/r05/g10; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
NNSP_LIB=abtest/split/nnsp_amd/libnnsp_mi355x.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_nnsp.py tests/test_gpu_cascade.py tests/test_gpu_benchloop.py tests/test_gpu_refnets.py tests/test_gpu_configs.py > $O/pytest_split.log 2>&1 || { echo "split pytest failed"; tail -40 $O/pytest_split.log; exit 1; }
tail -1 $O/pytest_split.log
bash profiles/r05/ab.sh NNSP_LIB "abtest/base/nnsp_amd/libnnsp_mi355x.so - abtest/split/nnsp_amd/libnnsp_mi355x.so" 3 || exit 1
for L in - abtest/split/nnsp_amd/libnnsp_mi355x.so; do if [ $L = - ]; then unset NNSP_LIB; else export NNSP_LIB=$L; fi; timeout -k 10 300 python bench.py --net s2i --no-cpu-baseline > $O/s2i_$(basename $(dirname $(dirname $L)) 2>/dev/null).json 2>>$O/s2i.err || { echo s2i failed; exit 1; }; done; unset NNSP_LIB
for f in $O/s2i_*.json; do python -c "import json; d=json.load(open('$f')); print('$f', round(d['value']/1e9,4), round(d['nn_ms_per_step'],4))"; done
echo all-ok
