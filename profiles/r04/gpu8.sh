#!/bin/bash
# bisect the cascade detected-mismatch over the three uncommitted changes (variant libraries)
set -o pipefail
O=gpurun_out/r04; mkdir -p $O
export TMPDIR=/tmp
chk() { if grep -q -i "illegal memory\|HSA_STATUS\|memory access fault" $1; then echo "GPU FAULT in $1"; tail -20 $1; exit 1; fi; }
for v in prev v_nosplit v_norecur v_noproj cur; do
  if [ $v = cur ]; then unset NNSP_LIB; else export NNSP_LIB=abtest/$v/nnsp_amd/libnnsp_mi355x.so; fi
  timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu "tests/test_gpu_cascade.py::test_cascade_matches_oracle" > $O/bisect8_$v.log 2>&1; rc=$?; chk $O/bisect8_$v.log; [ $rc -le 1 ] || exit 1
  echo "$v: $(tail -1 $O/bisect8_$v.log)"
done
unset NNSP_LIB
timeout -k 10 300 python -u profiles/r04/diag_benchcfg.py ref > $O/diag8_default.log 2>&1; rc=$?; chk $O/diag8_default.log; [ $rc -le 1 ] || exit 1
grep -v "^    " $O/diag8_default.log | tail -12; grep "^    " $O/diag8_default.log | head -14
echo diag-done
