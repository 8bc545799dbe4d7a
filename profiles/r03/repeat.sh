#!/bin/bash
# the default bench line five times on one box (spread of the headline)
set -o pipefail
mkdir -p gpurun_out/r03/rep
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --no-stress > gpurun_out/r03/rep/b$i.json 2> gpurun_out/r03/rep/b$i.err || { echo "bench $i failed"; tail -5 gpurun_out/r03/rep/b$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03/rep/b$i.json')); print($i, round(d['value']/1e9,4), round(d['ms_per_step'],3), round(d['fe_ms_per_step'],3))"
done
