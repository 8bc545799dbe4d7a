#!/bin/bash
# round 6: Mel bank index in the LDS tables (no batch-mode spill), staging loads behind the tables' -- full GPU
# suite (required), drop-in clocks and latency, single-net (batch front end) and cascade A/B against h6
set -o pipefail
O=gpurun_out/r06/${TAG:-g22}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_all.log 2>&1 || { echo "pytest (required) failed"; tail -40 $O/pytest_all.log; exit 1; }
tail -1 $O/pytest_all.log
NNSP_LIB=abtest/p6/nnsp_amd/libnnsp_mi355x.so timeout -k 10 120 python profiles/r06/dropin_probe.py > $O/probe.txt 2>&1 || { echo "probe failed"; tail -20 $O/probe.txt; exit 1; }
grep -v "^   L" $O/probe.txt
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --dropin-latency > $O/lat_$rep.json 2> $O/lat_$rep.err || { echo "latency failed"; tail -20 $O/lat_$rep.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/lat_$rep.json').read().strip().split('\n')[-1])
print('rep $rep', {k:(round(v['gpu_us_per_frame_median'],1), round(v['gpu_us_per_frame_p99'],1)) for k,v in d['nets'].items()})"
done
bash profiles/r06/ab.sh NNSP_LIB "abtest/h6/nnsp_amd/libnnsp_mi355x.so -" 3 --net vad || exit 1
mv gpurun_out/r06/ab_NNSP_LIB $O/ab_vad
bash profiles/r06/ab.sh NNSP_LIB "abtest/h6/nnsp_amd/libnnsp_mi355x.so -" 3 || exit 1
mv gpurun_out/r06/ab_NNSP_LIB $O/ab_cascade
echo all-ok
