#!/bin/bash
# final round-4 records: PMC profile of the default cascade bench (kernel trace + stats, one pass per
# counter group), its summary as the bench's profile, default bench x3, configs[1..3], the
# ARM_OPTIMIZED=0 build, strong scaling on one GPU, drop-in latency
set -o pipefail
O=gpurun_out/r04/final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_final.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_final.log; exit 1; }
tail -1 $O/pytest_final.log
bash profiles/r04/prof.sh $O/cascade || exit 1
python3 profiles/r04/summarize.py $O/cascade cascade 32768 100 ref mix $O/pmc_cascade.json > $O/summ.log 2>&1 || { echo "summarize failed"; tail -5 $O/summ.log; exit 1; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --profile-json $O/pmc_cascade.json > $O/bench_cascade_$i.json 2> $O/bench_cascade_$i.err || { echo "bench $i failed"; tail -5 $O/bench_cascade_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_cascade_$i.json')); print('cascade', round(d['value']/1e9,4), round(d['ms_per_step'],3), d['roofline'].get('frac'), d['roofline'].get('valu_busy'), d.get('cascade_synthetic_weights',{}).get('value'))"
done
for net in vad kws s2i; do
  timeout -k 10 300 python bench.py --net $net > $O/bench_$net.json 2> $O/bench_$net.err || { echo "bench $net failed"; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$net.json')); print('$net', round(d['value']/1e9,4), round(d['ms_per_step'],3))"
done
timeout -k 10 300 python bench.py --net s2i --acc32 --no-cpu-baseline > $O/bench_s2i_acc32.json 2> $O/bench_s2i_acc32.err || { echo "bench s2i acc32 failed"; exit 1; }
timeout -k 10 300 python bench.py --build portable --no-cpu-baseline > $O/bench_portable.json 2> $O/bench_portable.err || { echo "bench portable failed"; exit 1; }
timeout -k 10 300 python bench.py --scaling strong --steps 5 --no-cpu-baseline --no-stress > $O/bench_strong_n1.json 2> $O/bench_strong.err || { echo "bench strong failed"; exit 1; }
timeout -k 10 300 python bench.py --dropin-latency > $O/dropin.json 2> $O/dropin.err || { echo "dropin failed"; exit 1; }
for f in s2i_acc32 portable strong_n1; do python -c "import json; d=json.load(open('$O/bench_$f.json')); print('$f', round(d['value']/1e9,4), round(d['ms_per_step'],3))"; done
echo all-ok
