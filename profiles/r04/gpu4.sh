#!/bin/bash
# drop-in single-copy frame + prebuilt tables; round 0 launched before the behind-the-fork copies
set -o pipefail
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu4.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu4.log; exit 1; }
tail -1 $O/pytest_gpu4.log
timeout -k 10 300 python bench.py --dropin-latency > $O/dropin4.json 2> $O/dropin4.err || { echo "dropin failed"; tail -10 $O/dropin4.err; exit 1; }
python -c "import json; d=json.load(open('$O/dropin4.json'))['nets']; print({k:(round(v['gpu_us_per_frame_median'],1), round(v['cpu_baseline']['us_per_frame'],2)) for k,v in d.items()})"
bash profiles/r04/ab.sh NNSP_LIB "abtest/prev/nnsp_amd/libnnsp_mi355x.so -" 4
