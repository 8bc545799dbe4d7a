#!/bin/bash
# kernel trace of the default bench (final build: stream-ordering events without timestamps): per-chunk timeline
set -o pipefail
O=gpurun_out/r05/g52; mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --no-stress --steps 6 --warmup 2"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- $B > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1)
python3 profiles/r03/chunk_timeline.py $f 3 > $O/timeline.txt || exit 1
echo all-ok
