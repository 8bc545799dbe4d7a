#!/bin/bash
# diagnose the bench-config cascade mismatch: where, and with the multi-tile recur off
set -o pipefail
O=gpurun_out/r04; mkdir -p $O
export TMPDIR=/tmp
chk() { if grep -q -i "illegal memory\|HSA_STATUS\|memory access fault" $1; then echo "GPU FAULT in $1"; tail -20 $1; exit 1; fi; }
timeout -k 10 300 python -u profiles/r04/diag_benchcfg.py ref > $O/diag7_default.log 2>&1; rc=$?; chk $O/diag7_default.log; [ $rc -le 1 ] || exit 1
grep -v "^    " $O/diag7_default.log | tail -12; grep "^    " $O/diag7_default.log | head -14
NNSP_RECUR_TSEQ=1 timeout -k 10 300 python -u profiles/r04/diag_benchcfg.py ref > $O/diag7_tseq1.log 2>&1; rc=$?; chk $O/diag7_tseq1.log; [ $rc -le 1 ] || exit 1
grep -v "^    " $O/diag7_tseq1.log | tail -8
NNSP_LIB=abtest/prev/nnsp_amd/libnnsp_mi355x.so timeout -k 10 300 python -u profiles/r04/diag_benchcfg.py ref > $O/diag7_prev.log 2>&1; rc=$?; chk $O/diag7_prev.log; [ $rc -le 1 ] || exit 1
grep -v "^    " $O/diag7_prev.log | tail -8
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_nnsp.py tests/test_gpu_cascade.py > $O/pytest7.log 2>&1; rc=$?; chk $O/pytest7.log; [ $rc -le 1 ] || exit 1
tail -15 $O/pytest7.log
echo diag-done
