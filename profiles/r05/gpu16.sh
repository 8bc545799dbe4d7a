#!/bin/bash
# shared front end schedules (NNSP_FE_SCHED): 0 equal ranges, 1 guided (default), 2 per-XCD blocks with a share
set -o pipefail
O=gpurun_out/r05/g16; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_benchloop.py tests/test_gpu_cascade.py tests/test_gpu_bigshard.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash profiles/r05/ab2.sh fesched2 "NNSP_FE_SCHED=0 NNSP_FE_SCHED=1 NNSP_FE_SCHED=2" 4 || exit 1
for V in 0 1; do
  env NNSP_FE_GENS=5 NNSP_FE_SCHED=$V NNSP_LIB=abtest/probes2/nnsp_amd/libnnsp_mi355x.so timeout -k 10 200 python profiles/r03/wg_timeline.py 32768 $O/wg_$V.npz > $O/wg_$V.txt 2>&1 || { echo "wg_timeline failed"; tail -5 $O/wg_$V.txt; exit 1; }
done
echo all-ok
