#!/bin/bash
# when the look-ahead front end starts (NNSP_AHEAD_MODE 0: after round 0; 1: after round 1's proj;
# 2: after round 1): parity with mode 1, A/B, kernel trace of mode 1
set -o pipefail
O=gpurun_out/r04/g19; mkdir -p $O
export TMPDIR=/tmp
NNSP_AHEAD_MODE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_cascade.py tests/test_gpu_benchcfg.py > $O/pytest19_m1.log 2>&1 || { echo "pytest mode 1 failed"; tail -30 $O/pytest19_m1.log; exit 1; }
tail -1 $O/pytest19_m1.log
bash profiles/r04/ab.sh NNSP_AHEAD_MODE "0 1 2" 2 --no-cpu-baseline || exit 1
NNSP_AHEAD_MODE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_m1 -o kt -- python3 bench.py --no-cpu-baseline --no-stress --steps 3 --warmup 1 > $O/kt_m1.log 2>&1 || { echo "trace failed"; exit 1; }
echo all-ok
