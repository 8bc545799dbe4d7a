#!/bin/bash
# round 6: fused VAD prefix -- stage clocks (PROBES build) with and without fusion; kernel trace of a fused bench
set -o pipefail
O=gpurun_out/r06/g5; mkdir -p $O
export TMPDIR=/tmp
for F in 0 1; do
  NNSP_LIB=abtest/p6/nnsp_amd/libnnsp_mi355x.so NNSP_FUSE_PREFIX=$F timeout -k 10 200 python profiles/r06/casc_clocks_fp.py > $O/clk_$F.txt 2>&1 || { echo "clocks $F failed"; tail -20 $O/clk_$F.txt; exit 1; }
  cat $O/clk_$F.txt
done
NNSP_FUSE_PREFIX=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o kt -- python3 bench.py --no-cpu-baseline --no-stress --steps 4 --warmup 2 > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1)
python3 profiles/r03/chunk_timeline.py $f 2 > $O/timeline.txt || exit 1
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    agg[r["Kernel_Name"][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
keys = [k for k in rows[0].keys() if "LDS" in k or "VGPR" in k or "Scratch" in k]
seen = set()
for r in rows:
    k = r["Kernel_Name"][:60]
    if "recur_pipe" in k and k not in seen:
        seen.add(k)
        print(k, {kk: r[kk] for kk in keys}, "n", len(agg[k]), "mean us", round(sum(agg[k]) / len(agg[k]), 1))
PY
echo all-ok
