#!/bin/bash
# full GPU suite + smoke + default bench line
set -o pipefail
mkdir -p gpurun_out/r03
T=${TAG:-full}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03/${T}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r03/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/r03/${T}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03/${T}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r03/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/r03/${T}_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r03/${T}_bench.json 2> gpurun_out/r03/${T}_bench.err || { echo "bench failed"; tail -20 gpurun_out/r03/${T}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r03/${T}_bench.json')); print(d['value']/1e9, d['ms_per_step'], d['fe_ms_per_step'])"
