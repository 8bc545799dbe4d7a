#!/bin/bash
# after the post-wave changes: per-stage recurrence clocks and the round-0 workgroup timeline (PROBES build),
# a kernel trace of the default bench
set -o pipefail
O=gpurun_out/r05/g9; mkdir -p $O
export TMPDIR=/tmp
NNSP_LIB=abtest/probes/nnsp_amd/libnnsp_mi355x.so timeout -k 10 200 python profiles/r02/casc_clocks.py > $O/casc_clocks.txt 2>&1 || { echo "casc_clocks failed"; tail -5 $O/casc_clocks.txt; exit 1; }
grep -v amdgpu.ids $O/casc_clocks.txt
NNSP_LIB=abtest/probes/nnsp_amd/libnnsp_mi355x.so timeout -k 10 200 python profiles/r03/wg_timeline.py 32768 $O/wg.npz > $O/wg_timeline.txt 2>&1 || { echo "wg_timeline failed"; tail -5 $O/wg_timeline.txt; exit 1; }
head -42 $O/wg_timeline.txt | grep -v amdgpu.ids
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --no-cpu-baseline --no-stress --steps 5 --warmup 2 > $O/kt.log 2>&1 || { echo "kt failed"; tail -5 $O/kt.log; exit 1; }
echo all-ok
