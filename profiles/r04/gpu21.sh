#!/bin/bash
# final round-4 records, part 2: suite, default bench x3 (profile of part 1), configs[1..3]
set -o pipefail
O=gpurun_out/r04/final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_final.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_final.log; exit 1; }
tail -1 $O/pytest_final.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py > $O/bench_default_$i.json 2> $O/bench_default_$i.err || { echo "bench $i failed"; tail -5 $O/bench_default_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_default_$i.json')); r=d['roofline']; print('cascade', round(d['value']/1e9,4), round(d['ms_per_step'],3), round(r.get('frac'),3), r.get('valu_busy'), d.get('cascade_synthetic_weights',{}).get('value'), d['cpu_baseline']['value'])"
done
for net in vad kws s2i; do
  timeout -k 10 300 python bench.py --net $net > $O/bench_$net.json 2> $O/bench_$net.err || { echo "bench $net failed"; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$net.json')); print('$net', round(d['value']/1e9,4), round(d['ms_per_step'],3), d['cpu_baseline']['value'])"
done
echo all-ok
