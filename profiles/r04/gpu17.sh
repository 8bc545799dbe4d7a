#!/bin/bash
# FC epilogue constants folded into the accumulators (proj prefix layer and recur FC stages, ACC32),
# log10 with 24-bit multiplies: suite, per-stage clocks and A/B against af60ab8's parent build (r4b)
set -o pipefail
O=gpurun_out/r04/g17; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest17.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest17.log; exit 1; }
tail -1 $O/pytest17.log
for v in r4b cur; do
  if [ $v = cur ]; then unset NNSP_LIB; else export NNSP_LIB=abtest/$v/nnsp_amd/libnnsp_mi355x.so; fi
  for net in s2i kws vad; do
    timeout -k 10 120 python profiles/recur_clocks.py $net 8192 ref > $O/clk_${v}_$net.log 2>&1 || { echo "clocks $v $net failed"; exit 1; }
    echo "$v $net: $(grep -v amdgpu.ids $O/clk_${v}_$net.log | head -6 | tr '\n' ' ' | cut -c1-330)"
  done
done
unset NNSP_LIB
for net in s2i kws vad; do
  bash profiles/r04/ab.sh NNSP_LIB "abtest/r4b/nnsp_amd/libnnsp_mi355x.so -" 2 --net $net --no-stress || exit 1
done
bash profiles/r04/ab.sh NNSP_LIB "abtest/r4b/nnsp_amd/libnnsp_mi355x.so -" 3 || exit 1
echo all-ok
