#!/bin/bash
# recur: several tiles per workgroup through one pipeline (tseq); proj descriptor pipeline
# through LDS-DMA; split with opaque rounded products.  Suite, A/B against HEAD's build,
# tseq sweep, kernel traces of the reference and synthetic-weight cascades.
set -o pipefail
O=gpurun_out/r04; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_nnsp.py -k back_to_back > $O/pytest_gpu6a.log 2>&1 || { echo "focused pytest failed"; tail -30 $O/pytest_gpu6a.log; exit 1; }
tail -1 $O/pytest_gpu6a.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu6.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu6.log; exit 1; }
tail -1 $O/pytest_gpu6.log
bash profiles/r04/ab.sh NNSP_LIB "abtest/prev/nnsp_amd/libnnsp_mi355x.so -" 3 || exit 1
bash profiles/r04/ab.sh NNSP_RECUR_TSEQ "1 2 4" 2 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_ref6 -o kt -- python3 bench.py --no-cpu-baseline --no-stress --steps 3 --warmup 1 > $O/kt_ref6.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_synth6 -o kt -- python3 bench.py --no-cpu-baseline --no-stress --weights synth --steps 3 --warmup 1 > $O/kt_synth6.log 2>&1 || { echo "synth trace failed"; exit 1; }
timeout -k 10 300 python bench.py --dropin-latency > $O/dropin6.json 2> $O/dropin6.err || { echo "dropin failed"; tail -10 $O/dropin6.err; exit 1; }
python -c "import json; d=json.load(open('$O/dropin6.json'))['nets']; print({k:(round(v['gpu_us_per_frame_median'],1), round(v['cpu_baseline']['us_per_frame'],2)) for k,v in d.items()})"
echo all-ok
