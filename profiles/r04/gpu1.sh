#!/bin/bash
# round 4, first GPU pass: full GPU suite (incl. the >2^32 ring-offset cascades),
# default bench, strong-scaling shard (262144 streams) on one GPU
set -o pipefail
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
timeout -k 10 400 python bench.py --scaling strong --no-stress --no-cpu-baseline --steps 5 > $O/bench_strong_n1.json 2> $O/bench_strong_n1.err || { echo "strong bench failed"; tail -20 $O/bench_strong_n1.err; exit 1; }
python -c "
import json
for f in ('bench_default','bench_strong_n1'):
    d=json.load(open('$O/'+f+'.json')); print(f, d['value']/1e9, 'G', d['ms_per_step'], 'ms', d['roofline']['frac'], d.get('cascade_synthetic_weights',{}).get('value',0)/1e9)
"
