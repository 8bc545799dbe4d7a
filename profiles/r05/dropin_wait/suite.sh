#!/bin/bash
# the GPU suite, smoke and two drop-in latency records with the completion-word wait (default)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/g44
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --dropin-latency > $O/dropin_$i.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
done
python - <<'PY'
import json
for i in (1, 2):
    d = json.load(open(f"gpurun_out/r05/g44/dropin_{i}.json"))["nets"]
    print(i, {n: (round(v["gpu_us_per_frame_median"], 2), round(v["gpu_us_per_frame_p99"], 1), round(v["cpu_baseline"]["us_per_frame"], 2)) for n, v in d.items()})
PY
echo all-ok
