#!/bin/bash
# casc_begin split over the nets' streams: kernel-trace timeline with it on, then a second paired A/B
set -o pipefail
O=gpurun_out/r05/g46; mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --no-cpu-baseline --no-stress --steps 6 --warmup 2"
export NNSP_BEGIN_SPLIT=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- $B > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
unset NNSP_BEGIN_SPLIT
f=$(find $O/kt -name '*kernel_trace.csv' | head -1)
python3 profiles/r03/chunk_timeline.py $f 3 > $O/timeline.txt || exit 1
head -40 $O/timeline.txt
bash profiles/r05/ab2.sh bsplit2 "- NNSP_BEGIN_SPLIT=1" 5 || exit 1
echo all-ok
