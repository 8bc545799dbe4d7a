#!/bin/bash
# VAD's round-0 recurrence on a CU subset (NNSP_VAD_FREE CUs left to S2I / KWS): parity, then paired A/B
set -o pipefail
mkdir -p gpurun_out/r03
NNSP_VAD_FREE=${PT_FREE:-96} timeout -k 10 400 python -u -m pytest tests/test_gpu_cascade.py tests/test_gpu_benchcfg.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/vf_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03/vf_pytest.log; exit 1; }
tail -2 gpurun_out/r03/vf_pytest.log
bash profiles/r03/ab.sh NNSP_VAD_FREE "${VALS:-- 64 96 112 128}" ${REPS:-2}
