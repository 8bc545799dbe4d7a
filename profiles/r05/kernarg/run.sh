#!/bin/bash
# kernel arguments in device memory (HIP_FORCE_DEV_KERNARG=1) vs the runtime's default: drop-in latency, paired
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/kernarg; mkdir -p $O
for i in 1 2 3; do
  for w in 0 1; do
    timeout -k 10 200 env HIP_FORCE_DEV_KERNARG=$w python bench.py --dropin-latency --no-cpu-baseline > $O/k${w}_$i.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  done
done
python - <<'PY'
import json
for w in (0, 1):
    for i in (1, 2, 3):
        d = json.load(open(f"gpurun_out/r05/kernarg/k{w}_{i}.json"))["nets"]
        print(w, i, {n: (round(v["gpu_us_per_frame_median"], 2), round(v["gpu_us_per_frame_p99"], 1)) for n, v in d.items()})
PY
echo all-ok
