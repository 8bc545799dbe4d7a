#!/bin/bash
# round 6: drop-in weight staging loads behind the front end's table loads or after its prologue
# (NNSP_DROPIN_EARLY 1 / 0) -- parity (required), clocks, paired latency
set -o pipefail
O=gpurun_out/r06/${TAG:-g23}; mkdir -p $O
export TMPDIR=/tmp
for v in 1 0; do
NNSP_DROPIN_EARLY=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_legacy.py > $O/pytest_req_$v.log 2>&1 || { echo "pytest (required) failed"; tail -40 $O/pytest_req_$v.log; exit 1; }
tail -1 $O/pytest_req_$v.log
done
for v in 1 0; do
  NNSP_DROPIN_EARLY=$v NNSP_LIB=abtest/p6/nnsp_amd/libnnsp_mi355x.so timeout -k 10 120 python profiles/r06/dropin_probe.py > $O/probe_$v.txt 2>&1 || { echo "probe failed"; tail -20 $O/probe_$v.txt; exit 1; }
  echo "EARLY=$v"; grep "kernel phases" $O/probe_$v.txt | cut -c1-170
done
for rep in 1 2 3; do for v in 1 0; do
  NNSP_DROPIN_EARLY=$v timeout -k 10 200 python bench.py --dropin-latency > $O/lat_${v}_$rep.json 2> $O/lat_${v}_$rep.err || { echo "latency failed"; tail -20 $O/lat_${v}_$rep.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/lat_${v}_$rep.json').read().strip().split('\n')[-1])
print('EARLY=$v rep $rep', {k:(round(v['gpu_us_per_frame_median'],1), round(v['gpu_us_per_frame_p99'],1)) for k,v in d['nets'].items()})"
done; done
echo all-ok
