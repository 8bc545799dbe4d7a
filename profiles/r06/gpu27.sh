#!/bin/bash
# round 6: drop-in: wave 0's front-end frame at issue priority 3 over the staging waves (NNSP_DI_PRIO) -- parity of
# the variant (required), clocks, paired latency
set -o pipefail
O=gpurun_out/r06/${TAG:-g27}; mkdir -p $O
export TMPDIR=/tmp
NNSP_LIB=abtest/pr1/nnsp_amd/libnnsp_mi355x.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_legacy.py > $O/pytest_req.log 2>&1 || { echo "pytest (required) failed"; tail -40 $O/pytest_req.log; exit 1; }
tail -1 $O/pytest_req.log
for v in p8 ppr1; do
  NNSP_LIB=abtest/$v/nnsp_amd/libnnsp_mi355x.so timeout -k 10 120 python profiles/r06/dropin_probe.py > $O/probe_$v.txt 2>&1 || { echo "probe failed"; tail -20 $O/probe_$v.txt; exit 1; }
  echo "$v"; grep "kernel phases" $O/probe_$v.txt | cut -c60-330
done
for rep in 1 2 3; do for v in base pr1; do
  if [ $v = pr1 ]; then export NNSP_LIB=abtest/pr1/nnsp_amd/libnnsp_mi355x.so; else unset NNSP_LIB; fi
  timeout -k 10 200 python bench.py --dropin-latency > $O/lat_${v}_$rep.json 2> $O/lat_${v}_$rep.err || { echo "latency failed"; tail -20 $O/lat_${v}_$rep.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/lat_${v}_$rep.json').read().strip().split('\n')[-1])
print('$v rep $rep', {k:(round(v['gpu_us_per_frame_median'],1), round(v['gpu_us_per_frame_p99'],1)) for k,v in d['nets'].items()})"
done; done
unset NNSP_LIB
echo all-ok
