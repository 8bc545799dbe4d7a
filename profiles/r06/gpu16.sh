#!/bin/bash
# round 6: drop-in host-side phases beside the kernel's
set -o pipefail
O=gpurun_out/r06/${TAG:-g16}; mkdir -p $O
export TMPDIR=/tmp
NNSP_LIB=abtest/p6/nnsp_amd/libnnsp_mi355x.so timeout -k 10 120 python profiles/r06/dropin_probe.py > $O/probe.txt 2>&1 || { echo "probe failed"; tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt
echo all-ok
