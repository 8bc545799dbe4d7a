#!/bin/bash
# round-4 final records (FE tail, bank sums, addresses), part 1: full GPU suite, PMC profile of the
# default cascade bench, its summary, default bench x3
set -o pipefail
O=gpurun_out/r04/final3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_final.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_final.log; exit 1; }
tail -1 $O/pytest_final.log
bash profiles/r04/prof.sh $O/cascade || exit 1
python3 profiles/r04/summarize.py $O/cascade cascade 32768 100 ref mix $O/pmc_cascade.json > $O/summ.log 2>&1 || { echo "summarize failed"; tail -5 $O/summ.log; exit 1; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --profile-json $O/pmc_cascade.json > $O/bench_cascade_$i.json 2> $O/bench_cascade_$i.err || { echo "bench $i failed"; tail -5 $O/bench_cascade_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_cascade_$i.json')); r=d['roofline']; print('cascade', round(d['value']/1e9,4), round(d['ms_per_step'],3), round(r.get('frac'),3), r.get('valu_busy'), r.get('traffic'), d.get('cascade_synthetic_weights',{}).get('value'), d['cpu_baseline']['value'])"
done
echo all-ok
