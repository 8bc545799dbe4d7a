#!/bin/bash
# FE counter passes on the cascade bench (one rocprofv3 run per pass), per
# shared-FE kernel name.  usage: fe_pmc.sh OUTDIR [env assignments...]
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=$1; shift
for kv in "$@"; do export "$kv"; done
mkdir -p $D
B="python3 bench.py --no-cpu-baseline --no-stress --steps 3 --warmup 1"
R="--kernel-include-regex fe_kernel --output-format csv"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
P3="SQ_ACTIVE_INST_SALU SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_LDS_ADDR_CONFLICT"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P $R -d $D/p$i -o p$i -- $B > $D/p$i.log 2>&1 || { echo "pass $i rc=$?"; tail -3 $D/p$i.log; exit 1; }
done
python3 - "$D" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(collections.Counter)
for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name", "")
        if "fe_kernel" not in k: continue
        if "ILi2E" in k or "<2" in k: continue   # cold front end
        k = k.split("(")[0]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]] += 1
for k in tot:
    print(k)
    for c in sorted(tot[k]): print(f"  {c:28s} {tot[k][c]/max(1,n[k][c]):.4g}  (n={n[k][c]})")
PY
