#!/bin/bash
# paired A/B over environment settings on one box: ab2.sh NAME "S1 S2 ..." [reps] [bench args]
# a setting is "-" (nothing set) or K=V[+K2=V2...]; the summary is ab.sh's
set -o pipefail
NAME=$1; VALS=$2; REPS=${3:-4}; shift 3; ARGS="$*"
O=gpurun_out/r05/ab_${NAME}
mkdir -p $O
for i in $(seq $REPS); do
  j=0
  for V in $VALS; do
    j=$((j+1))
    ENVS=()
    if [ "$V" != "-" ]; then IFS='+' read -ra ENVS <<< "$V"; fi
    timeout -k 10 300 env "${ENVS[@]}" python bench.py --no-cpu-baseline $ARGS > $O/${j}_$i.json 2> $O/err.log || { echo "bench $V failed"; tail -5 $O/err.log; exit 1; }
  done
done
python - "$O" "$VALS" "$REPS" <<'PY'
import json, sys, statistics as st
o, vals, reps = sys.argv[1], sys.argv[2].split(), int(sys.argv[3])
for j, v in enumerate(vals, 1):
    ds = [json.load(open(f"{o}/{j}_{i}.json")) for i in range(1, reps + 1)]
    med = lambda xs: round(st.median(xs), 4)
    xs = [d["value"] / 1e9 for d in ds]
    line = {"setting": v[-60:], "G": med(xs), "runs": [round(x, 4) for x in xs], "fe_ms": med([d["fe_ms_per_step"] for d in ds]),
            "ms_step": med([d["ms_per_step"] for d in ds])}
    if "cascade_synthetic_weights" in ds[0]:
        line["synth_G"] = med([d["cascade_synthetic_weights"]["value"] / 1e9 for d in ds])
    print(json.dumps(line))
PY
