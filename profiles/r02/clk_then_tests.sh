#!/bin/bash
# recur clocks for each variant (s2i, kws; reference nets), then the GPU suite
set -u
cd $GRAFT_REPO_ROOT
for v in $VARIANTS; do
  for n in s2i kws; do
    echo "== $v $n"; NNSP_LIB=abtest/$v/nnsp_amd/libnnsp_mi355x.so timeout -k 10 120 python -u profiles/recur_clocks.py $n 8192 ref || exit 4
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; exit $rc
