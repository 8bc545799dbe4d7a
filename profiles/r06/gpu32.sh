#!/bin/bash
# round 6: diagnose test_nnsp_exec_tables_rewritten_in_place on the new build and on w3 (HEAD)
set -o pipefail
O=gpurun_out/r06/${TAG:-g32}; mkdir -p $O
export TMPDIR=/tmp
for v in new w3; do
  if [ $v = new ]; then unset NNSP_LIB; else export NNSP_LIB=abtest/$v/nnsp_amd/libnnsp_mi355x.so; fi
  timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_legacy.py -k "rewritten or generic_nets" > $O/pytest_$v.log 2>&1; echo "$v rc=$?"
  grep -h "passed\|failed\|net: LSTM\|frame" $O/pytest_$v.log | head -6
  NNSP_DROPIN_WORKER=0 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_legacy.py -k "rewritten" > $O/pytest_${v}_w0.log 2>&1; echo "$v worker0 rc=$?"
  grep -h "passed\|failed\|net: LSTM" $O/pytest_${v}_w0.log | head -4
done
echo all-ok
