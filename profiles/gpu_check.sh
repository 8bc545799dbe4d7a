#!/bin/bash
# GPU parity tests + a short bench of the three nets (used during development)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
for n in vad kws s2i; do
  timeout -k 10 200 python bench.py --net $n --no-cpu-baseline > gpurun_out/bench_$n.json 2> gpurun_out/bench_$n.err || { echo "bench $n failed"; tail -5 gpurun_out/bench_$n.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$n.json'));print('$n',round(d['value']/1e6,1),'Mfr/s',d['kernels_ms_per_step'])"
done
