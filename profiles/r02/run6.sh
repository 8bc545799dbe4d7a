#!/bin/bash
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_nnsp.py tests/test_gpu_refnets.py -k "vad or n3" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run() { n=$1; shift; timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-stress "$@" > $O/b_$n.json 2>> $O/bench.err || exit 4; }
run vad --net vad
run ref
run synth --weights synth
echo done
