#!/bin/bash
# Round-3 final records: PART=tests (GPU suite + smoke), PART=prof W... (kernel trace + PMC passes of each
# workload, summarised), PART=bench W... (bench lines with the matching PMC summary).  Output: gpurun_out/r03f
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03f
mkdir -p $O
PART=$1; shift
args_of() { [ "$1" = cascade ] && echo "" || echo "--net $1"; }
streams_of() { [ "$1" = cascade ] && echo 32768 || echo 8192; }
case $PART in
tests)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 \
    || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log ;;
prof)
  for W in "$@"; do
    bash profiles/r02/prof.sh $O/$W $(args_of $W) || exit 1
    python3 profiles/r02/summarize.py $O/$W $W $(streams_of $W) 100 ref mix $O/${W}_summary.json || exit 1
    echo "prof $W ok"
  done ;;
bench)
  for W in "$@"; do
    X=""; T=$W
    case $W in *_acc32) X="--acc32"; W=${W%_acc32};; esac
    timeout -k 10 400 python bench.py $(args_of $W) $X --profile-json $O/${W}_summary.json > $O/bench_$T.json 2> $O/bench_$T.err \
      || { echo "bench $T failed"; tail -20 $O/bench_$T.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$O/bench_$T.json')); print('$T', round(d['value']/1e9,4), 'G', round(d['ms_per_step'],3), 'ms', 'frac', round(d['roofline']['frac'],3), 'traffic', d['roofline']['traffic'])"
  done ;;
esac
