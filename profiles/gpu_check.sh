#!/bin/bash
# Development GPU check: parity tests, then short benches.  Stops at the first
# crash / timeout (exit status other than 0 or 1 from pytest).
#   usage: profiles/gpu_check.sh [pytest -k expr] [bench nets...]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K=${1:-}
shift || true
NETS=${@:-cascade vad kws s2i}
timeout -k 10 500 python -m pytest tests -m gpu -x -q ${K:+-k "$K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for n in $NETS; do
  timeout -k 10 300 python bench.py --net $n --no-cpu-baseline > gpurun_out/bench_$n.json 2> gpurun_out/bench_$n.err || { echo "bench $n failed"; tail -5 gpurun_out/bench_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$n.json'));print('$n',round(d['value']/1e6,2),'Mfr/s',d['kernels_ms_per_step'],d.get('cascade'),d['roofline']['kernel'],round(d['roofline']['frac'],3))"
done
