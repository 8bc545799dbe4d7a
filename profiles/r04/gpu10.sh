#!/bin/bash
# S2I's instrumented NN time rose 0.32 -> 0.59 ms in the cascade A/B: single-net A/B and the
# per-stage recur clocks, prev (HEAD) vs current build
set -o pipefail
O=gpurun_out/r04; mkdir -p $O
export TMPDIR=/tmp
for net in s2i kws vad; do
  bash profiles/r04/ab.sh NNSP_LIB "abtest/prev/nnsp_amd/libnnsp_mi355x.so -" 2 --net $net --no-stress || exit 1
done
for v in prev cur; do
  if [ $v = cur ]; then unset NNSP_LIB; else export NNSP_LIB=abtest/prev/nnsp_amd/libnnsp_mi355x.so; fi
  for net in s2i kws vad; do
    timeout -k 10 120 python profiles/recur_clocks.py $net 8192 ref > $O/clk10_${v}_$net.log 2>&1 || { echo "clocks $v $net failed"; tail -5 $O/clk10_${v}_$net.log; exit 1; }
    echo "$v $net: $(head -8 $O/clk10_${v}_$net.log | tr '\n' ' ')"
  done
done
unset NNSP_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_s2i10 -o kt -- python3 bench.py --no-cpu-baseline --net s2i --steps 3 --warmup 1 > $O/kt_s2i10.log 2>&1 || { echo "trace failed"; exit 1; }
echo all-ok
