cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for B in 4096 4608 3072 6144; do
  for n in cascade vad; do
    NNSP_FE_BLOCKS=$B timeout -k 10 200 python bench.py --net $n --no-cpu-baseline > gpurun_out/sw_${n}_$B.json 2>gpurun_out/sw.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/sw_${n}_$B.json'));print('$B $n',round(d['value']/1e6,1),d['kernels_ms_per_step'])"
  done
done
