#!/bin/bash
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUTD:-r02q1}
mkdir -p $O
NNSP_CASCADE_DEBUG=1 timeout -k 10 120 python -u profiles/r02/bisect_casc.py > $O/small.log 2>&1 || { tail -5 $O/small.log; exit 3; }
tail -1 $O/small.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
OUTD=${OUTD:-r02q1} bash profiles/r02/sweep_ahead.sh
