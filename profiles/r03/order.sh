#!/bin/bash
# round-0 launch-order A/B (NNSP_R0_ORDER): bench + workgroup timeline per order
set -o pipefail
mkdir -p gpurun_out/r03/order
for O in 0 1 3 0 1 3 3; do
  export NNSP_R0_ORDER=$O
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-stress > gpurun_out/r03/order/b$O.json 2> gpurun_out/r03/order/err.log || { echo "bench $O failed"; tail -5 gpurun_out/r03/order/err.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03/order/b$O.json')); print('order $O', round(d['value']/1e6,1), round(d['ms_per_step'],3))"
done
for O in 3; do
  export NNSP_R0_ORDER=$O
  timeout -k 10 200 python -u profiles/r03/wg_timeline.py 32768 > gpurun_out/r03/order/wg$O.txt 2>&1 || { tail -5 gpurun_out/r03/order/wg$O.txt; exit 1; }
  head -10 gpurun_out/r03/order/wg$O.txt | tail -8
done
