#!/bin/bash
# FE phase clocks (single-net VAD) and one SQ counter pass over the VAD bench
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${OUTD:-r02fe}
mkdir -p $O
timeout -k 10 120 python3 profiles/recur_clocks.py vad 32768 > $O/clk_vad.log 2>&1 || { tail -5 $O/clk_vad.log; exit 3; }
grep -v amdgpu.ids $O/clk_vad.log
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_VALU -d $O/pmc -o pmc -- python3 bench.py --no-cpu-baseline --no-stress --net vad --steps 3 --warmup 1 > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 4; }
echo pmc-ok
