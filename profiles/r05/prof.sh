#!/bin/bash
# Round-4 profile of one bench configuration: kernel trace + stats, then one
# rocprofv3 --pmc pass per counter group (FETCH_SIZE and WRITE_SIZE in passes
# of their own, MI355X_MICROARCH.md; <= 8 SQ counters and GRBM per pass).
# usage: profiles/r04/prof.sh OUTDIR [bench args...]
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=$1; shift
mkdir -p $D
B="python3 bench.py --no-cpu-baseline --no-stress --steps 3 --warmup 1 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o kt -- $B > $D/kt.log 2>&1 \
    || { echo "kt failed"; tail -5 $D/kt.log; exit 1; }
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $D/p$i -o p$i -- $B > $D/p$i.log 2>&1 \
      || { echo "pass $i ($P) rc=$?"; tail -3 $D/p$i.log; exit 2; }
done
echo prof-ok
