#!/bin/bash
# small cascade check, the GPU suite, benches, and a profile of the default bench
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02r
mkdir -p $O
NNSP_CASCADE_DEBUG=1 timeout -k 10 120 python -u profiles/r02/bisect_casc.py > $O/small.log 2>&1 || { tail -5 $O/small.log; exit 3; }
tail -1 $O/small.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
grep -q "Error 700\|illegal memory" $O/pytest.log && exit 5
run() { n=$1; shift; timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-stress "$@" > $O/b_$n.json 2>> $O/bench.err || exit 4; }
run ref
run synth --weights synth
run vad --net vad
bash profiles/r02/prof.sh $O/cascade_ref
echo done
