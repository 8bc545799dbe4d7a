#!/bin/bash
# One SQ counter pass (+ GRBM clock) over the cascade bench; the shared front end's rows
# are summarised by profiles/r02/pmc_rows.py.  usage: profiles/r02/fe_pmc2.sh OUTDIR
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=$1
mkdir -p $O
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/p -o p -- python3 bench.py --no-cpu-baseline --no-stress --steps 3 --warmup 1 > $O/p.log 2>&1 || { tail -5 $O/p.log; exit 4; }
echo pmc-ok
