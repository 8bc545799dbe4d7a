#!/bin/bash
# kernel trace of a short bench run (timeline analysis: profiles/r02/timeline.py)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/${OUTD:-r02v}
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/kt -o kt -- python3 bench.py --no-cpu-baseline --no-stress --steps 4 --warmup 1 "$@" > $D/kt.log 2>&1 || { tail -5 $D/kt.log; exit 1; }
echo trace-ok
