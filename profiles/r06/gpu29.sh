#!/bin/bash
# round 6: resident drop-in worker with its staging before the request loop (the loop body without it) --
# parity (required), worker / one-launch clocks, paired latency against the first worker build (w1)
set -o pipefail
O=gpurun_out/r06/${TAG:-g29}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_legacy.py > $O/pytest_req.log 2>&1 || { echo "pytest (required) failed"; tail -40 $O/pytest_req.log; exit 1; }
tail -1 $O/pytest_req.log
for v in 1 0; do
  NNSP_DROPIN_WORKER=$v NNSP_LIB=abtest/p9/nnsp_amd/libnnsp_mi355x.so timeout -k 10 120 python profiles/r06/dropin_probe.py > $O/probe_w$v.txt 2>&1 || { echo "probe failed"; tail -20 $O/probe_w$v.txt; exit 1; }
  echo "WORKER=$v"; grep "host:\|kernel phases" $O/probe_w$v.txt | cut -c1-330
done
for rep in 1 2 3; do for v in w1 new; do
  if [ $v = w1 ]; then export NNSP_LIB=abtest/w1/nnsp_amd/libnnsp_mi355x.so; else unset NNSP_LIB; fi
  timeout -k 10 200 python bench.py --dropin-latency > $O/lat_${v}_$rep.json 2> $O/lat_${v}_$rep.err || { echo "latency failed"; tail -20 $O/lat_${v}_$rep.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/lat_${v}_$rep.json').read().strip().split('\n')[-1])
print('$v rep $rep', {k:(round(v['gpu_us_per_frame_median'],1), round(v['gpu_us_per_frame_p99'],1)) for k,v in d['nets'].items()})"
done; done
unset NNSP_LIB
echo all-ok
