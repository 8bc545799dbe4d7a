#!/bin/bash
# shared front end with dynamic frame blocks (FeArgs.tickets, default) vs static ranges (NNSP_FE_DYN=0):
# cascade suites, paired A/B, and the round-0 + front-end wave timeline (PROBES build)
set -o pipefail
O=gpurun_out/r05/g14; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cascade.py tests/test_gpu_benchloop.py tests/test_gpu_cascade_state.py tests/test_gpu_benchcfg.py tests/test_gpu_shards.py tests/test_gpu_bigshard.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash profiles/r05/ab.sh NNSP_FE_DYN "0 -" 3 || exit 1
NNSP_LIB=abtest/probes2/nnsp_amd/libnnsp_mi355x.so timeout -k 10 200 python profiles/r03/wg_timeline.py 32768 $O/wg.npz > $O/wg_timeline.txt 2>&1 || { echo "wg_timeline failed"; tail -5 $O/wg_timeline.txt; exit 1; }
head -12 $O/wg_timeline.txt | grep -v amdgpu.ids
echo all-ok
