#!/bin/bash
# round 6: drop-in inputs in the kernel arguments (NNSP_DROPIN_KARG) -- parity (required), clocks, paired latency
set -o pipefail
O=gpurun_out/r06/${TAG:-g20}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_legacy.py tests/test_gpu_legacy_portable.py tests/test_gpu_nnsp_e2e.py tests/test_gpu_refnets.py > $O/pytest_req.log 2>&1 || { echo "pytest (required) failed"; tail -40 $O/pytest_req.log; exit 1; }
tail -1 $O/pytest_req.log
for v in 1 0; do
  NNSP_DROPIN_KARG=$v NNSP_LIB=abtest/p6/nnsp_amd/libnnsp_mi355x.so timeout -k 10 120 python profiles/r06/dropin_probe.py > $O/probe_$v.txt 2>&1 || { echo "probe failed"; tail -20 $O/probe_$v.txt; exit 1; }
  echo "KARG=$v"; grep -v "^   L" $O/probe_$v.txt
done
for rep in 1 2 3; do for v in 1 0; do
  NNSP_DROPIN_KARG=$v timeout -k 10 200 python bench.py --dropin-latency > $O/lat_${v}_$rep.json 2> $O/lat_${v}_$rep.err || { echo "latency failed"; tail -20 $O/lat_${v}_$rep.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/lat_${v}_$rep.json').read().strip().split('\n')[-1])
print('KARG=$v rep $rep', {k:(round(v['gpu_us_per_frame_median'],1), round(v['gpu_us_per_frame_p99'],1)) for k,v in d['nets'].items()})"
done; done
echo all-ok
