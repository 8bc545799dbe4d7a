#!/bin/bash
# round 6: drop-in out of LDS + phased epilogue + staged activation table; front end's batched
# table load and lane-index image -- full GPU suite (required), drop-in clocks / latency, headline A/B
set -o pipefail
O=gpurun_out/r06/${TAG:-g14}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_all.log 2>&1 || { echo "pytest (required) failed"; tail -40 $O/pytest_all.log; exit 1; }
tail -1 $O/pytest_all.log
NNSP_LIB=abtest/p6/nnsp_amd/libnnsp_mi355x.so timeout -k 10 120 python profiles/r06/dropin_probe.py > $O/probe.txt 2>&1 || { echo "probe failed"; tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt
timeout -k 10 200 python bench.py --dropin-latency > $O/lat.json 2> $O/lat.err || { echo "latency failed"; tail -20 $O/lat.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/lat.json').read().strip().split('\n')[-1])
print({k:(round(v['gpu_us_per_frame_median'],1), round(v['gpu_us_per_frame_p99'],1)) for k,v in d['nets'].items()})"
bash profiles/r06/ab.sh NNSP_LIB "abtest/h6/nnsp_amd/libnnsp_mi355x.so -" 3 || exit 1
echo all-ok
