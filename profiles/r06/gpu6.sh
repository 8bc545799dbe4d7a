#!/bin/bash
# round 6: fused VAD prefix -- the prefix wave's sub-phase clocks (PROBES build)
set -o pipefail
O=gpurun_out/r06/g6; mkdir -p $O
NNSP_LIB=abtest/p6/nnsp_amd/libnnsp_mi355x.so NNSP_FUSE_PREFIX=1 timeout -k 10 200 python profiles/r06/casc_clocks_fp.py > $O/clk_1.txt 2>&1 || { echo "clocks failed"; tail -20 $O/clk_1.txt; exit 1; }
cat $O/clk_1.txt
echo all-ok
