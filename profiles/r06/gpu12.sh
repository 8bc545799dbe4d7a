#!/bin/bash
# round 6: drop-in phase clocks kept in LDS (no per-phase mapped-memory store)
set -o pipefail
O=gpurun_out/r06/${TAG:-g12}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_legacy.py tests/test_gpu_refnets.py > $O/pytest_req.log 2>&1 || { echo "pytest (required) failed"; tail -40 $O/pytest_req.log; exit 1; }
tail -1 $O/pytest_req.log

for v in 1 0; do
  NNSP_DROPIN_LDS=$v NNSP_LIB=abtest/p6/nnsp_amd/libnnsp_mi355x.so timeout -k 10 120 python profiles/r06/dropin_probe.py > $O/probe_$v.txt 2>&1 || { echo "probe failed"; tail -20 $O/probe_$v.txt; exit 1; }
  echo "LDS=$v"; cat $O/probe_$v.txt
done
echo all-ok
