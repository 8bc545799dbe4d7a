#!/bin/bash
# drop-in call: the layers' A fragments staged in LDS (NNSP_DROPIN_STAGE, default on) -- legacy and refnet GPU
# suites, then paired latency runs off / on
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05/stage
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_legacy.py tests/test_gpu_legacy_portable.py tests/test_gpu_refnets.py tests/test_gpu_nnsp_e2e.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2 3; do
  for w in 0 1; do
    timeout -k 10 200 env NNSP_DROPIN_STAGE=$w python bench.py --dropin-latency --no-cpu-baseline > $O/s${w}_$i.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  done
done
python - <<'PY'
import json
for w in (0, 1):
    for i in (1, 2, 3):
        d = json.load(open(f"gpurun_out/r05/stage/s{w}_{i}.json"))["nets"]
        print(w, i, {n: (round(v["gpu_us_per_frame_median"], 2), round(v["gpu_us_per_frame_p99"], 1)) for n, v in d.items()})
PY
echo all-ok
