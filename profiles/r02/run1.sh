#!/bin/bash
# second round-2 GPU call: the fixed tests, then kernel traces of the cascade
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_refnets.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash profiles/r02/prof.sh $O/w0 --window 0 && bash profiles/r02/prof.sh $O/w16 && bash profiles/r02/prof.sh $O/synth --weights synth
