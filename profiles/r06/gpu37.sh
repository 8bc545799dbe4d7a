#!/bin/bash
# round 6: drop-in FC layers of <= 4 row tiles on one wave, no barrier between two (NNSP_DI_W0) -- parity (required: legacy + e2e), paired latency vs w0off
set -o pipefail
O=gpurun_out/r06/${TAG:-g37}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_legacy.py tests/test_gpu_nnsp_e2e.py > $O/pytest_req.log 2>&1 || { echo "pytest (required) failed"; tail -40 $O/pytest_req.log; exit 1; }
tail -1 $O/pytest_req.log
for rep in 1 2 3; do for v in w0off new; do
  if [ $v = new ]; then unset NNSP_LIB; else export NNSP_LIB=abtest/$v/nnsp_amd/libnnsp_mi355x.so; fi
  timeout -k 10 200 python bench.py --dropin-latency > $O/lat_${v}_$rep.json 2> $O/lat_${v}_$rep.err || { echo "latency failed"; tail -20 $O/lat_${v}_$rep.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/lat_${v}_$rep.json').read().strip().split('\n')[-1])
print('$v rep $rep', {k:(round(v['gpu_us_per_frame_median'],1), round(v['gpu_us_per_frame_p99'],1)) for k,v in d['nets'].items()})"
done; done
unset NNSP_LIB
echo all-ok
