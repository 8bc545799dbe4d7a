#!/bin/bash
# kernel trace of a short default bench run (timeline: profiles/r02/timeline.py TRACE.csv)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUTD:-r03/kt}
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D -o kt -- python3 bench.py --no-cpu-baseline --no-stress --steps 6 --warmup 2 "$@" > $D/kt.log 2>&1 || { tail -5 $D/kt.log; exit 1; }
find $D -name "*kernel_trace.csv" | head -3
echo trace-ok
