#!/bin/bash
# paired A/B of an environment setting on one box: ab.sh VAR "A B" [reps] [bench args] -- bench lines per setting
set -o pipefail
VAR=$1; VALS=$2; REPS=${3:-6}; shift 3; ARGS="$*"
mkdir -p gpurun_out/r03/ab
for i in $(seq $REPS); do
  j=0
  for V in $VALS; do
    j=$((j+1))
    if [ "$V" = "-" ]; then unset $VAR; else export $VAR=$V; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-stress $ARGS > gpurun_out/r03/ab/${VAR}_${j}_$i.json 2> gpurun_out/r03/ab/err.log || { echo "bench $V failed"; tail -5 gpurun_out/r03/ab/err.log; exit 1; }
  done
done
python - "$VAR" "$VALS" "$REPS" <<'PY'
import json, sys, statistics as st
var, vals, reps = sys.argv[1], sys.argv[2].split(), int(sys.argv[3])
for j, v in enumerate(vals, 1):
    ds = [json.load(open(f"gpurun_out/r03/ab/{var}_{j}_{i}.json")) for i in range(1, reps + 1)]
    xs = [d["value"] / 1e6 for d in ds]
    fe = [d.get("fe_ms_per_step", 0) for d in ds]
    nn = [sum((d.get("nn_ms_per_step") or {}).values()) if isinstance(d.get("nn_ms_per_step"), dict) else (d.get("nn_ms_per_step") or 0) for d in ds]
    print(var, v[-40:], "median", round(st.median(xs), 1), "fe_ms", round(st.median(fe), 3), "nn_ms", round(st.median(nn), 3), "runs", [round(x, 1) for x in xs])
PY
