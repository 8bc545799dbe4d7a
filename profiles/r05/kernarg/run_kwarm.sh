#!/bin/bash
# drop-in call: the NN's kernel arguments loaded before the front end (NNSP_DROPIN_KWARM, default on) -- legacy
# GPU suites, then paired latency runs off / on
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/kwarm2; mkdir -p $O
true
true
for i in 1 2 3 4 5 6; do
  for w in 0 1; do
    timeout -k 10 200 env NNSP_DROPIN_KWARM=$w python bench.py --dropin-latency --no-cpu-baseline > $O/w${w}_$i.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  done
done
python - <<'PY'
import json
for w in (0, 1):
    for i in (1, 2, 3, 4, 5, 6):
        d = json.load(open(f"gpurun_out/r05/kwarm2/w{w}_{i}.json"))["nets"]
        print(w, i, {n: (round(v["gpu_us_per_frame_median"], 2), round(v["gpu_us_per_frame_p99"], 1)) for n, v in d.items()})
PY
echo all-ok
