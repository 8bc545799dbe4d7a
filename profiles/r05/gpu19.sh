#!/bin/bash
# kernel traces of the default bench and of NNSP_EARLY_RETURN=1: per-chunk timelines (the gap between the
# look-ahead front end's end and the next chunk's first kernel)
set -o pipefail
O=gpurun_out/r05/g19; mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --no-stress --steps 6 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt0 -o kt -- $B > $O/kt0.log 2>&1 || { echo "kt0 failed"; tail -5 $O/kt0.log; exit 1; }
NNSP_EARLY_RETURN=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt1 -o kt -- $B > $O/kt1.log 2>&1 || { echo "kt1 failed"; tail -5 $O/kt1.log; exit 1; }
for k in kt0 kt1; do
  f=$(find $O/$k -name '*kernel_trace.csv' | head -1)
  python3 profiles/r03/chunk_timeline.py $f 3 > $O/$k.txt || exit 1
done
echo all-ok
