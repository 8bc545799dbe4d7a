#!/bin/bash
# drop-in input copy overlapped with the front end's table staging: suites, drop-in latency, VAD bench
set -o pipefail
O=gpurun_out/r05/g39; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --dropin-latency > $O/dropin_$i.json 2> $O/dropin.err || { echo "dropin failed"; tail -10 $O/dropin.err; exit 1; }
  python -c "import json; d=json.load(open('$O/dropin_$i.json'))['nets']; print({k:(round(v['gpu_us_per_frame_median'],1), round(v['gpu_us_per_frame_p99'],1)) for k,v in d.items()})"
done
timeout -k 10 300 python bench.py --net vad --no-cpu-baseline > $O/bench_vad.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_vad.json')); print('vad', round(d['value']/1e9,4))"
echo all-ok
