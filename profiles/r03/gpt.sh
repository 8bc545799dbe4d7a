#!/bin/bash
# proj tiles of 2 / 4 streams for long segments (NNSP_PROJ_GPT): parity at both, then paired A/B (cascade and VAD)
set -o pipefail
mkdir -p gpurun_out/r03
for G in 2 4; do
  NNSP_PROJ_GPT=$G timeout -k 10 600 python -u -m pytest tests/test_gpu_cascade.py tests/test_gpu_benchcfg.py tests/test_gpu_nnsp.py tests/test_gpu_refnets.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/gpt_pytest_$G.log 2>&1 || { echo "pytest G=$G failed"; tail -30 gpurun_out/r03/gpt_pytest_$G.log; exit 1; }
  tail -1 gpurun_out/r03/gpt_pytest_$G.log
done
bash profiles/r03/ab.sh NNSP_PROJ_GPT "- 2 4" 3 && bash profiles/r03/ab.sh NNSP_PROJ_GPT "- 2 4" 2 --net vad
