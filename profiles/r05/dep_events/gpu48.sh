#!/bin/bash
# stream-ordering events without timestamps: stress-case timeline with them on, then a second paired A/B
set -o pipefail
O=gpurun_out/r05/g48; mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --no-stress --weights synth --steps 6 --warmup 2"
export NNSP_DEP_EVENTS=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- $B > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
unset NNSP_DEP_EVENTS
f=$(find $O/kt -name '*kernel_trace.csv' | head -1)
python3 profiles/r03/chunk_timeline.py $f 2 > $O/timeline_synth.txt || exit 1
bash profiles/r05/ab2.sh depev2 "- NNSP_DEP_EVENTS=1" 6 || exit 1
echo all-ok
