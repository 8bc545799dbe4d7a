#!/bin/bash
# full GPU suite on the guided front-end schedule, then two default benches
set -o pipefail
O=gpurun_out/r05/g18; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do timeout -k 10 300 python bench.py > $O/bench_$i.json 2> $O/bench_err.log || { echo "bench failed"; tail -5 $O/bench_err.log; exit 1; }; done
python -c "
import json
for i in (1, 2):
    d = json.load(open('$O/bench_%d.json' % i)); print(round(d['value'] / 1e9, 4), d['ms_per_step'], d['fe_ms_per_step'])"
echo all-ok
