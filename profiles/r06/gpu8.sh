#!/bin/bash
# round 6: proj_kernel phase clocks (PROBES build), VAD and KWS single-net batches
set -o pipefail
O=gpurun_out/r06/g8; mkdir -p $O
for n in vad kws; do
  NNSP_LIB=abtest/p6/nnsp_amd/libnnsp_mi355x.so timeout -k 10 200 python profiles/proj_clocks.py $n 32768 100 > $O/proj_$n.txt 2>&1 || { echo "proj clocks failed"; tail -20 $O/proj_$n.txt; exit 1; }
  cat $O/proj_$n.txt
done
echo all-ok
