#!/bin/bash
# Counter passes (one rocprofv3 run per pass) of one kernel (regex KRE, default fe_kernel) on a
# single-net bench.  usage: profiles/fe_pmc.sh [net] [out-dir]
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
NET=${1:-vad}
D=${2:-gpurun_out/fepmc}
mkdir -p $D
B="python3 bench.py --net $NET --no-cpu-baseline --steps 3 --warmup 1"
R="--kernel-include-regex ${KRE:-fe_kernel} --output-format csv"
timeout -k 10 120 rocprofv3 -L > $D/counters.txt 2>&1 || echo "list rc=$?"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
P3="SQ_ACTIVE_INST_SALU SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_LDS_ADDR_CONFLICT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P $R -d $D/p$i -o p$i -- $B > $D/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 $D/p$i.log; }
done
python3 - "$D" <<'PY'
import csv, glob, sys, collections, os
d = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if os.environ.get("KRE", "fe_kernel").split("|")[0] not in r.get("Kernel_Name", ""): continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
for k in sorted(tot): print(f"{k:28s} {tot[k]/max(1,n[k]):.4g}  (n={n[k]})")
PY
