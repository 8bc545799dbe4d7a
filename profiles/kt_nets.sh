#!/bin/bash
# Kernel-trace stats of the single-net benches and the cascade (one rocprofv3 run each).
#   usage: profiles/kt_nets.sh [workloads...]   (default: vad kws s2i cascade)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for n in ${@:-vad kws s2i cascade}; do
  D=gpurun_out/kt_$n
  mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o kt -- python3 bench.py --net $n --no-cpu-baseline --steps 5 --warmup 1 > $D/bench.json 2> $D/err.log || { echo "$n failed"; tail -3 $D/err.log; exit 1; }
  python3 - $D <<'PY'
import csv, sys
d = sys.argv[1]
rows = list(csv.DictReader(open(f"{d}/kt_kernel_stats.csv")))
print(d)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f"  {r['Name'][:58]:58s} n={r['Calls']:>5s} avg={float(r['AverageNs'])/1e3:9.1f}us tot={float(r['TotalDurationNs'])/1e6:8.2f}ms")
PY
done
