#!/bin/bash
# final round-4 records, part 1: PMC profile of the default cascade bench (kernel trace + stats, one
# pass per counter group), its summary as the bench's profile, the default bench twice
set -o pipefail
O=gpurun_out/r04/final; mkdir -p $O
export TMPDIR=/tmp
bash profiles/r04/prof.sh $O/cascade || exit 1
python3 profiles/r04/summarize.py $O/cascade cascade 32768 100 ref mix $O/pmc_cascade.json > $O/summ.log 2>&1 || { echo "summarize failed"; tail -5 $O/summ.log; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --profile-json $O/pmc_cascade.json > $O/bench_cascade_$i.json 2> $O/bench_cascade_$i.err || { echo "bench $i failed"; tail -5 $O/bench_cascade_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_cascade_$i.json')); r=d['roofline']; print('cascade', round(d['value']/1e9,4), round(d['ms_per_step'],3), r.get('frac'), r.get('valu_busy'), r.get('traffic'), d.get('cascade_synthetic_weights',{}).get('value'))"
done
echo all-ok
