#!/bin/bash
# round-2 GPU call 3: cascade tests (look-ahead, auto window), then the bench
# with / without the look-ahead front end, ref and synth weights
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_cascade.py tests/test_gpu_benchcfg.py tests/test_gpu_shards.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for cfg in "ref" "ref --no-lookahead" "synth" "synth --no-lookahead" "ref --window 0" "synth --window 16"; do
  set -- $cfg
  n=$(echo "$cfg" | tr ' ' '_' | tr -d '-')
  timeout -k 10 200 python -u bench.py --weights $cfg --no-cpu-baseline --no-stress > $O/bench_$n.json 2>> $O/bench.err || exit 4
done
echo done
