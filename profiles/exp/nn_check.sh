# parity of the batch + cascade paths, stage clocks, then the four benches
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_nnsp.py tests/test_gpu_cascade.py > gpurun_out/nn_check.log 2>&1 || { tail -30 gpurun_out/nn_check.log; exit 1; }
tail -1 gpurun_out/nn_check.log
for n in ${CLK:-vad kws s2i}; do timeout -k 10 100 python3 profiles/recur_clocks.py $n 8192 || exit 1; done
for n in ${NETS:-vad kws s2i cascade}; do
  timeout -k 10 200 python3 bench.py --net $n --no-cpu-baseline > gpurun_out/nc_$n.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/nc_$n.json')); print('$n', round(d['value']/1e6,1), {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
done
