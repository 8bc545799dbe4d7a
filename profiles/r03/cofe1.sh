#!/bin/bash
# co-running front end (NNSP_COFE) parity on the look-ahead test, then a paired A/B of settings
set -o pipefail
mkdir -p gpurun_out/r03
NNSP_COFE=${PT_COFE:-3,64,25,6,1} timeout -k 10 300 python -u -m pytest tests/test_gpu_cascade.py -k "lookahead or stats" -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/cofe_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03/cofe_pytest.log; exit 1; }
tail -2 gpurun_out/r03/cofe_pytest.log
bash profiles/r03/ab.sh NNSP_COFE "${VALS:-- 3,64,25,6,0 3,64,25,6,1 2,64,25,6,1 3,32,25,6,1 3,128,25,6,1}" ${REPS:-2}
