#!/bin/bash
# per-net tiles per workgroup for short segments (VAD 4, S2I / KWS 2): full GPU suite, smoke(), A/B against
# HEAD's build (r4h) on the synthetic-weight line and the headline, 3 passes each
set -o pipefail
O=gpurun_out/r04/g44; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest44.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest44.log; exit 1; }
tail -1 $O/pytest44.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash profiles/r04/ab.sh NNSP_LIB "abtest/r4h/nnsp_amd/libnnsp_mi355x.so -" 3 --weights synth --no-stress || exit 1
bash profiles/r04/ab.sh NNSP_LIB "abtest/r4h/nnsp_amd/libnnsp_mi355x.so -" 3 --no-stress || exit 1
echo all-ok
