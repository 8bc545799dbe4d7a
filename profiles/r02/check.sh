#!/bin/bash
# Round-2 GPU check: the GPU parity suite, the default bench line, and a
# cascade window sweep on the reference nets.  usage: profiles/r02/check.sh OUT
set -u
cd $GRAFT_REPO_ROOT
O=${1:-gpurun_out/r02}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread \
    > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc     # 1 = test failures (keep going), else a crash / timeout
timeout -k 10 300 python -u bench.py --cpu-seconds 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 3; }
for w in 0 8 24; do
  timeout -k 10 200 python -u bench.py --window $w --no-cpu-baseline --no-stress > $O/bench_w$w.json 2>> $O/bench.err || exit 4
done
echo done
