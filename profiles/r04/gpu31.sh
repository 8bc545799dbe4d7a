#!/bin/bash
# synthetic-weight stress line: window sweep on the current build (auto = 16 frames per round at
# this cut rate; WS overrides the list), two passes
set -o pipefail
O=gpurun_out/r04/g31; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for W in ${WS:--1 24 32 48 0}; do
    timeout -k 10 300 python bench.py --weights synth --window $W --no-stress --no-cpu-baseline > $O/w${W}_$rep.json 2> $O/err.log || { echo "bench W=$W failed"; tail -5 $O/err.log; exit 1; }
    python -c "import json; d=json.load(open('$O/w${W}_$rep.json')); print('W', $W, round(d['value']/1e9,4), round(d['ms_per_step'],3))"
  done
done
echo all-ok
