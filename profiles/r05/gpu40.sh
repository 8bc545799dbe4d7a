#!/bin/bash
# the drop-in call in one launch (dropin_kernel): full GPU suite, drop-in latency, cascade and VAD benches
set -o pipefail
O=gpurun_out/r05/g40; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --dropin-latency > $O/dropin_$i.json 2> $O/dropin.err || { echo "dropin failed"; tail -10 $O/dropin.err; exit 1; }
  python -c "import json; d=json.load(open('$O/dropin_$i.json'))['nets']; print({k:(round(v['gpu_us_per_frame_median'],1), round(v['gpu_us_per_frame_p99'],1)) for k,v in d.items()})"
done
bash profiles/r05/ab2.sh fuse_check "- NNSP_FE_SCHED=1" 2 || exit 1
echo all-ok
