#!/bin/bash
# NN-kernel counter pass (proj / recur) on a bench line.  usage: nn_pmc.sh OUTDIR REGEX [bench args...]
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=$1; RX=$2; shift 2
mkdir -p $D
B="python3 bench.py --no-cpu-baseline --no-stress --steps 3 --warmup 1 $*"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA"
P2="GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$RX" --output-format csv -d $D/p$i -o p$i -- $B > $D/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 $D/p$i.log; exit 1; }
done
python3 - "$D" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(collections.Counter)
for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "").split("(")[0]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]] += 1
for k in tot:
    print(k[:100])
    for c in sorted(tot[k]): print(f"  {c:28s} {tot[k][c]/max(1,n[k][c]):.4g}  (n={n[k][c]})")
PY
