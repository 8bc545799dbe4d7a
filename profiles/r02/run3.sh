#!/bin/bash
# round-2 GPU call 4: look-ahead test; look-ahead scheduling knobs A/B (net
# stream priority, look-ahead front-end grid cap)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_cascade.py -k lookahead -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run() { n=$1; shift; env "$@" timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-stress > $O/b_$n.json 2>> $O/bench.err || exit 4; }
run base
run fpw4 NNSP_AHEAD_FE_FPW=4
run fpw8 NNSP_AHEAD_FE_FPW=8
run fpw16 NNSP_AHEAD_FE_FPW=16
run fpw32 NNSP_AHEAD_FE_FPW=32
run fpw8_normal NNSP_AHEAD_FE_FPW=8 NNSP_NET_PRIO_NORMAL=1
run base2
echo done
