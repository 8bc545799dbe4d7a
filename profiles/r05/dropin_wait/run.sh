#!/bin/bash
# drop-in call: how the host waits for its launch (NNSP_DROPIN_WAIT 0 stream sync, 1 stream polling, 2 the
# kernel's completion word) -- legacy GPU suites with 2, then paired latency runs 0 / 1 / 2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/wait
mkdir -p $O
timeout -k 10 300 env NNSP_DROPIN_WAIT=2 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_legacy.py tests/test_gpu_legacy_portable.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2 3; do
  for w in 0 1 2; do
    timeout -k 10 200 env NNSP_DROPIN_WAIT=$w python bench.py --dropin-latency --no-cpu-baseline > $O/w${w}_$i.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  done
done
python - <<'PY'
import json
for w in (0, 1, 2):
    for i in (1, 2, 3):
        d = json.load(open(f"gpurun_out/r05/wait/w{w}_{i}.json"))["nets"]
        print(w, i, {n: (round(v["gpu_us_per_frame_median"], 2), round(v["gpu_us_per_frame_p99"], 1)) for n, v in d.items()})
PY
echo all-ok
