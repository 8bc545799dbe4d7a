set -u
mkdir -p gpurun_out/$1
timeout -k 10 400 python -u -m pytest tests/test_gpu_cascade.py tests/test_gpu_benchcfg.py tests/test_gpu_nnsp.py tests/test_gpu_legacy.py -x -q --timeout 200 --timeout-method thread > gpurun_out/$1/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/$1/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-stress > gpurun_out/$1/bench$i.json 2> gpurun_out/$1/bench$i.err || { tail -5 gpurun_out/$1/bench$i.err; exit 5; }
 python3 -c "import json;d=json.loads(open('gpurun_out/$1/bench$i.json').read().strip().splitlines()[-1]);print('casc',round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['fe_ms_per_step'],3), round(d['roofline']['frac'],4))"
done
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-stress --net vad > gpurun_out/$1/vad.json 2> gpurun_out/$1/vad.err || { tail -5 gpurun_out/$1/vad.err; exit 6; }
python3 -c "import json;d=json.loads(open('gpurun_out/$1/vad.json').read().strip().splitlines()[-1]);print('vad',round(d['value']/1e6,1), round(d['ms_per_step'],3), d.get('fe_ms_per_step'), round(d['roofline']['frac'],4))"
