#!/bin/bash
# drop-in call: inputs / results through mapped host memory inside the kernels (default) vs the two copies
# (NNSP_DROPIN_COPY=1); full GPU suite
set -o pipefail
O=gpurun_out/r05/g38; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  NNSP_DROPIN_COPY=1 timeout -k 10 300 python bench.py --dropin-latency > $O/dropin_copy_$i.json 2> $O/dropin.err || { echo "dropin copy failed"; tail -10 $O/dropin.err; exit 1; }
  timeout -k 10 300 python bench.py --dropin-latency > $O/dropin_map_$i.json 2> $O/dropin.err || { echo "dropin map failed"; tail -10 $O/dropin.err; exit 1; }
done
for f in $O/dropin_*.json; do python -c "import json; d=json.load(open('$f'))['nets']; print('$f'.split('/')[-1], {k:(round(v['gpu_us_per_frame_median'],1), round(v['gpu_us_per_frame_p99'],1)) for k,v in d.items()})"; done
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('cascade', round(d['value']/1e9,4), round(d['fe_ms_per_step'],3))"
echo all-ok
