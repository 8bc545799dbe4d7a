#!/bin/bash
# kernel trace of the drop-in latency bench: per-frame kernel durations
set -o pipefail
O=gpurun_out/r05/g34b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --dropin-latency > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
f=$(find $O/kt -name '*kernel_stats.csv' | head -1)
cut -d, -f1-8 $f | head -20
echo all-ok
