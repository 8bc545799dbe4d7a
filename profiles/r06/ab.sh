#!/bin/bash
# paired A/B on one box: ab.sh VAR "A B" [reps] [bench args]; "-" unsets VAR.
# Summary per setting: median frames/s, shared FE ms, instrumented per-net NN ms,
# synthetic-weight stress line (when the bench ran it)
set -o pipefail
VAR=$1; VALS=$2; REPS=${3:-4}; shift 3; ARGS="$*"
O=gpurun_out/r06/ab_${VAR}
mkdir -p $O
for i in $(seq $REPS); do
  j=0
  for V in $VALS; do
    j=$((j+1))
    if [ "$V" = "-" ]; then unset $VAR; else export $VAR=$V; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS > $O/${j}_$i.json 2> $O/err.log || { echo "bench $V failed"; tail -5 $O/err.log; exit 1; }
  done
done
unset $VAR
python - "$O" "$VALS" "$REPS" <<'PY'
import json, sys, statistics as st
o, vals, reps = sys.argv[1], sys.argv[2].split(), int(sys.argv[3])
for j, v in enumerate(vals, 1):
    ds = [json.load(open(f"{o}/{j}_{i}.json")) for i in range(1, reps + 1)]
    med = lambda xs: round(st.median(xs), 4)
    xs = [d["value"] / 1e9 for d in ds]
    line = {"setting": v[-50:], "G": med(xs), "runs": [round(x, 4) for x in xs], "fe_ms": med([d["fe_ms_per_step"] for d in ds]),
            "ms_step": med([d["ms_per_step"] for d in ds])}
    if "cascade" in ds[0]:
        for n in ("vad", "kws", "s2i"):
            line[n + "_nn_ms"] = med([d["cascade"]["instrumented_chunk"][n]["nn_ms"] for d in ds])
        if "cascade_synthetic_weights" in ds[0]:
            line["synth_G"] = med([d["cascade_synthetic_weights"]["value"] / 1e9 for d in ds])
    else:
        line["nn_ms"] = med([d["nn_ms_per_step"] for d in ds])
    print(json.dumps(line))
PY
