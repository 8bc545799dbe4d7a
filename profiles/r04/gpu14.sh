#!/bin/bash
# round 0's launch order (NNSP_R0_ORDER 0: VAD first, S2I/KWS NN wait for VAD's proj; 1: VAD first, no
# waits; 3: S2I and KWS first, VAD's recurrence waits for their proj) -- A/B and kernel traces
set -o pipefail
O=gpurun_out/r04/g14; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_benchcfg.py tests/test_gpu_cascade.py -k "bench_config or lookahead or matches_oracle" > $O/pytest14.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest14.log; exit 1; }
tail -1 $O/pytest14.log
NNSP_R0_ORDER=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_benchcfg.py tests/test_gpu_cascade.py -k "bench_config or lookahead or matches_oracle" > $O/pytest14_o3.log 2>&1 || { echo "pytest order 3 failed"; tail -30 $O/pytest14_o3.log; exit 1; }
tail -1 $O/pytest14_o3.log
bash profiles/r04/ab.sh NNSP_R0_ORDER "0 1 3" 3 || exit 1
for o in 1 3; do
  NNSP_R0_ORDER=$o timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_o$o -o kt -- python3 bench.py --no-cpu-baseline --no-stress --steps 3 --warmup 1 > $O/kt_o$o.log 2>&1 || { echo "trace $o failed"; exit 1; }
done
echo all-ok
