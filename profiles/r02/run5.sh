#!/bin/bash
# x-mode NN (proj hands x to recur): full GPU suite, then benches
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
run() { n=$1; shift; timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-stress "$@" > $O/b_$n.json 2>> $O/bench.err || exit 4; }
run ref
run ref_nolook --no-lookahead
run synth --weights synth
run vad --net vad
run kws --net kws
run s2i --net s2i
echo done
