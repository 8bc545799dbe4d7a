#!/bin/bash
# round 6: drop-in worker phase clocks with the device-memory mailbox (PROBES build p10)
set -o pipefail
O=gpurun_out/r06/${TAG:-g34}; mkdir -p $O
export TMPDIR=/tmp
NNSP_LIB=abtest/p10/nnsp_amd/libnnsp_mi355x.so timeout -k 10 120 python profiles/r06/dropin_probe.py > $O/probe_w1.txt 2>&1 || { echo "probe failed"; tail -20 $O/probe_w1.txt; exit 1; }
cat $O/probe_w1.txt | cut -c1-400
echo all-ok
