#!/bin/bash
# Refresh profiles/r01/<workload>/ for every bench workload, then the default bench line.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for w in cascade vad kws s2i; do
  bash profiles/collect_r01.sh $w > gpurun_out/coll_$w.log 2>&1 || { echo "collect $w failed"; tail -5 gpurun_out/coll_$w.log; exit 1; }
  echo "collected $w"
done
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
cat gpurun_out/bench_default.json
