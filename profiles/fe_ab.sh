#!/bin/bash
# FE change check: GPU parity tests, cascade + single-net benches, FE counters.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for n in cascade vad kws s2i; do
  timeout -k 10 200 python bench.py --net $n --no-cpu-baseline > gpurun_out/ab_$n.json 2>gpurun_out/ab.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$n.json'));print('$n',round(d['value']/1e6,1),d['kernels_ms_per_step'])"
done
bash profiles/fe_pmc.sh vad gpurun_out/fepmc_ab > gpurun_out/fepmc_ab.txt 2>&1 && grep -E "INSTS|BANK|WAVE_CYCLES" gpurun_out/fepmc_ab.txt
