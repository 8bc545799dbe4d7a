#!/bin/bash
# round 6, first GPU call: ADVICE fixes -- full GPU suite, smoke, two default benches
set -o pipefail
O=gpurun_out/r06/${TAG:-g1}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$i.json 2> $O/bench_$i.err || { echo "bench $i failed"; tail -5 $O/bench_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$i.json')); print('cascade', round(d['value']/1e9,4), round(d['ms_per_step'],3), round(d['fe_ms_per_step'],3), d.get('cascade_synthetic_weights',{}).get('value'))"
done
echo all-ok
