#!/bin/bash
# paired A/B of an environment setting on one box: ab.sh VAR "A B" [reps] -- bench lines per setting
set -o pipefail
VAR=$1; VALS=$2; REPS=${3:-6}
mkdir -p gpurun_out/r03/ab
for i in $(seq $REPS); do
  for V in $VALS; do
    if [ "$V" = "-" ]; then unset $VAR; else export $VAR=$V; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-stress > gpurun_out/r03/ab/${VAR}_${V}_$i.json 2> gpurun_out/r03/ab/err.log || { echo "bench $V failed"; tail -5 gpurun_out/r03/ab/err.log; exit 1; }
  done
done
python - "$VAR" "$VALS" "$REPS" <<'PY'
import json, sys, statistics as st
var, vals, reps = sys.argv[1], sys.argv[2].split(), int(sys.argv[3])
for v in vals:
    xs = [json.load(open(f"gpurun_out/r03/ab/{var}_{v}_{i}.json"))["value"] / 1e6 for i in range(1, reps + 1)]
    print(var, v, "median", round(st.median(xs), 1), "runs", [round(x, 1) for x in xs])
PY
