#!/bin/bash
# proj descriptor pipeline in LDS (asm LDS-DMA, fixed x-store count, parity-unrolled tile loop),
# drop-in single-copy frame, round 0 before the behind-the-fork copies
set -o pipefail
O=gpurun_out/r04; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu5.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu5.log; exit 1; }
tail -1 $O/pytest_gpu5.log
timeout -k 10 300 python bench.py --dropin-latency > $O/dropin5.json 2> $O/dropin5.err || { echo "dropin failed"; tail -10 $O/dropin5.err; exit 1; }
python -c "import json; d=json.load(open('$O/dropin5.json'))['nets']; print({k:(round(v['gpu_us_per_frame_median'],1), round(v['cpu_baseline']['us_per_frame'],2)) for k,v in d.items()})"
bash profiles/r04/ab.sh NNSP_LIB "abtest/prev/nnsp_amd/libnnsp_mi355x.so -" 4 || exit 1
bash profiles/r04/ab.sh NNSP_LIB "abtest/prev/nnsp_amd/libnnsp_mi355x.so -" 2 --net vad --no-stress || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_ref5 -o kt -- python3 bench.py --no-cpu-baseline --no-stress --steps 3 --warmup 1 > $O/kt_ref5.log 2>&1 || { echo "trace failed"; exit 1; }
echo trace-ok
