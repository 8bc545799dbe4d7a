#!/bin/bash
# six FE generations as the default: full GPU suite, smoke(), A/B against the eight-generation setting
# through the knob (same library), 3 passes
set -o pipefail
O=gpurun_out/r04/g41; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest41.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest41.log; exit 1; }
tail -1 $O/pytest41.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash profiles/r04/ab.sh NNSP_FE_GENS "- 8" 3 || exit 1
echo all-ok
