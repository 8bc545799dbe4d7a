#!/bin/bash
# round-0 dispatch: high-priority net streams (NNSP_NET_PRIO bitmask by NNSP_ID) x launch order
set -o pipefail
O=gpurun_out/r05/g5; mkdir -p $O
export TMPDIR=/tmp
bash profiles/r05/ab.sh NNSP_NET_PRIO "- 5 7 2" 2 || exit 1
export NNSP_NET_PRIO=5
bash profiles/r05/ab.sh NNSP_R0_ORDER "- 3 4" 2 || exit 1
export NNSP_LIB=abtest/probes/nnsp_amd/libnnsp_mi355x.so
timeout -k 10 200 python profiles/r03/wg_timeline.py 32768 $O/wg5.npz > $O/wg_timeline_prio5.txt 2>&1 || { echo "wg_timeline failed"; tail -5 $O/wg_timeline_prio5.txt; exit 1; }
head -40 $O/wg_timeline_prio5.txt
echo all-ok
