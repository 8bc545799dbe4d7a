#!/bin/bash
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_cascade.py -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run() { n=$1; shift; e=$1; shift; env $e timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-stress "$@" > $O/b_$n.json 2>> $O/bench.err || exit 4; }
run base NNSP_DUMMY=1
run nolook NNSP_DUMMY=1 --no-lookahead
run synth NNSP_DUMMY=1 --weights synth
run base2 NNSP_DUMMY=1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 bench.py --no-cpu-baseline --no-stress --steps 3 --warmup 1 > $O/kt.log 2>&1 || echo "kt rc=$?"
echo done
