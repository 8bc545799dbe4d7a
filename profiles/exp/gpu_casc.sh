cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_cascade.py > gpurun_out/casc_tests.log 2>&1 || { tail -30 gpurun_out/casc_tests.log; exit 1; }
tail -3 gpurun_out/casc_tests.log
timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 6 --warmup 2 > gpurun_out/casc_bench.json 2> gpurun_out/casc_bench.err || { tail -5 gpurun_out/casc_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/casc_bench.json')); print(round(d['value']/1e6,1), round(d['ms_per_step'],3), d.get('cascade'))"
