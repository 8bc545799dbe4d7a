#!/bin/bash
# recur: tile epilogues after the loop (no scratch, fewer SGPR spills), proj runtime-parity loop.
# Suite, per-stage clocks, A/B against HEAD's build (cascade + single nets)
set -o pipefail
O=gpurun_out/r04; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_cascade.py tests/test_gpu_nnsp.py > $O/pytest_gpu11a.log 2>&1 || { echo "focused pytest failed"; tail -30 $O/pytest_gpu11a.log; exit 1; }
tail -1 $O/pytest_gpu11a.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu11.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu11.log; exit 1; }
tail -1 $O/pytest_gpu11.log
for net in s2i kws vad; do
  timeout -k 10 120 python profiles/recur_clocks.py $net 8192 ref > $O/clk11_$net.log 2>&1 || { echo "clocks $net failed"; tail -5 $O/clk11_$net.log; exit 1; }
  echo "cur $net: $(grep -v amdgpu.ids $O/clk11_$net.log | head -7 | tr '\n' ' ')"
done
bash profiles/r04/ab.sh NNSP_LIB "abtest/prev/nnsp_amd/libnnsp_mi355x.so -" 3 || exit 1
for net in s2i kws vad; do
  bash profiles/r04/ab.sh NNSP_LIB "abtest/prev/nnsp_amd/libnnsp_mi355x.so -" 2 --net $net --no-stress || exit 1
done
echo all-ok
