#!/bin/bash
# short: suite on the current build (FC constants in the accumulators, log10 24-bit, ahead-mode knob)
set -o pipefail
O=gpurun_out/r04/g18; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest18.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest18.log; exit 1; }
tail -1 $O/pytest18.log
for v in r4b cur; do
  if [ $v = cur ]; then unset NNSP_LIB; else export NNSP_LIB=abtest/$v/nnsp_amd/libnnsp_mi355x.so; fi
  for net in s2i kws vad; do
    timeout -k 10 120 python profiles/recur_clocks.py $net 8192 ref > $O/clk_${v}_$net.log 2>&1 || { echo "clocks $v $net failed"; exit 1; }
    echo "$v $net: $(grep -v amdgpu.ids $O/clk_${v}_$net.log | head -6 | tr '\n' ' ' | cut -c1-330)"
  done
done
echo all-ok
