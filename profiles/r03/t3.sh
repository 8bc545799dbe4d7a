#!/bin/bash
# proj pipeline check: NN parity suites, then the default bench and the workgroup timeline
set -o pipefail
mkdir -p gpurun_out/r03
T=${TAG:-t3}
timeout -k 10 900 python -u -m pytest tests/test_gpu_nnsp.py tests/test_gpu_cascade.py tests/test_gpu_refnets.py tests/test_gpu_benchcfg.py tests/test_gpu_configs.py tests/test_gpu_shards.py tests/test_gpu_portable.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03/${T}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r03/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/r03/${T}_pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03/${T}_bench.json 2> gpurun_out/r03/${T}_bench.err || { echo "bench failed"; tail -20 gpurun_out/r03/${T}_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r03/${T}_bench.json')); print('bench', d['value']/1e9, d['ms_per_step'], d['fe_ms_per_step'])"
timeout -k 10 300 python -u profiles/r03/wg_timeline.py 32768 gpurun_out/r03/${T}_wg.npz > gpurun_out/r03/${T}_wg.txt 2>&1 || { tail -20 gpurun_out/r03/${T}_wg.txt; exit 1; }
head -10 gpurun_out/r03/${T}_wg.txt
