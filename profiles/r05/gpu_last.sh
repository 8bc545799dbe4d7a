#!/bin/bash
set -o pipefail
O=gpurun_out/r05/last; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -10 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(round(d['value']/1e9,4), d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
echo all-ok
