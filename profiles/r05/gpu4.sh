#!/bin/bash
# cell-state stride v2 (mod-32 banks): suite, A/B vs round start, LDS counters; round-0 probes (PROBES build)
set -o pipefail
O=gpurun_out/r05/g4; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash profiles/r05/ab.sh NNSP_LIB "abtest/base/nnsp_amd/libnnsp_mi355x.so -" 3 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o p -- python3 bench.py --no-cpu-baseline --no-stress --steps 3 --warmup 1 > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
export NNSP_LIB=abtest/probes/nnsp_amd/libnnsp_mi355x.so
timeout -k 10 200 python profiles/r02/casc_clocks.py > $O/casc_clocks.txt 2>&1 || { echo "casc_clocks failed"; tail -5 $O/casc_clocks.txt; exit 1; }
cat $O/casc_clocks.txt | tail -30
timeout -k 10 200 python profiles/r03/wg_timeline.py 32768 $O/wg.npz > $O/wg_timeline.txt 2>&1 || { echo "wg_timeline failed"; tail -5 $O/wg_timeline.txt; exit 1; }
head -60 $O/wg_timeline.txt
echo all-ok
