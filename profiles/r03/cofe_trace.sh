#!/bin/bash
# kernel traces of the bench with the co-running front end settings given (NNSP_COFE values; - = off)
set -o pipefail
export TMPDIR=/tmp
for V in ${VALS:-- 3,64,25,6,0}; do
  T=$(echo $V | tr ',' '_')
  VAR=${VAR:-NNSP_COFE}; if [ "$V" = "-" ]; then unset $VAR; else export $VAR=$V; fi
  D=gpurun_out/r03/ct_$T
  mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D -o kt -- python3 bench.py --no-cpu-baseline --no-stress --steps 6 --warmup 2 > $D/kt.log 2>&1 || { tail -5 $D/kt.log; exit 1; }
  F=$(find $D -name "*kernel_trace.csv" | head -1)
  python3 profiles/r03/chunk_timeline.py $F 1 > $D/timeline.txt
done
echo trace-ok
