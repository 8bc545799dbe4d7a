#!/bin/bash
# instruction-cache counters of recur_pipe_kernel, HEAD's build vs current (S2I and KWS single-net)
set -o pipefail
O=gpurun_out/r04/icache; mkdir -p $O
export TMPDIR=/tmp
for v in prev cur; do
  if [ $v = cur ]; then unset NNSP_LIB; else export NNSP_LIB=abtest/prev/nnsp_amd/libnnsp_mi355x.so; fi
  for net in s2i kws; do
    timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/${v}_$net -o p -- python3 bench.py --net $net --no-cpu-baseline --no-stress --steps 3 --warmup 1 > $O/${v}_$net.log 2>&1 || { echo "pmc $v $net rc=$?"; tail -5 $O/${v}_$net.log; exit 1; }
  done
done
unset NNSP_LIB
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/r04/icache/*/*counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].split("<")[0]
        agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
    for k in ("recur_pipe_kernel", "proj_kernel"):
        if k in agg: print(f.split("/")[-2], k, {c: round(v) for c, v in agg[k].items()})
PY
echo all-ok
