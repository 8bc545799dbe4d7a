#!/bin/bash
# drop-in NNSPClass_exec in place on mapped host memory (default) vs staged copies (NNSP_DROPIN_COPY=1)
set -o pipefail
O=gpurun_out/r05/g33; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_legacy.py tests/test_gpu_nnsp_e2e.py tests/test_gpu_legacy_portable.py tests/test_gpu_nnsp.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  NNSP_DROPIN_COPY=1 timeout -k 10 300 python bench.py --dropin-latency > $O/dropin_copy_$i.json 2> $O/dropin_copy.err || { echo "dropin copy failed"; tail -10 $O/dropin_copy.err; exit 1; }
  timeout -k 10 300 python bench.py --dropin-latency > $O/dropin_map_$i.json 2> $O/dropin_map.err || { echo "dropin map failed"; tail -10 $O/dropin_map.err; exit 1; }
done
for f in $O/dropin_*.json; do python -c "import json; d=json.load(open('$f'))['nets']; print('$f'.split('/')[-1], {k:(round(v['gpu_us_per_frame_median'],1), round(v['gpu_us_per_frame_p99'],1)) for k,v in d.items()})"; done
echo all-ok
