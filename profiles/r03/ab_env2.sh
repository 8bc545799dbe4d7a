#!/bin/bash
# parity of the cascade + batch suites with an env setting, then paired A/B: VAR VALS [REPS]
set -o pipefail
mkdir -p gpurun_out/r03
VAR=$1; VALS=$2; REPS=${3:-2}; PT=${PT:-1}
( [ "$PT" = "-" ] && unset $VAR || export $VAR=$PT; timeout -k 10 500 python -u -m pytest tests/test_gpu_cascade.py tests/test_gpu_benchcfg.py tests/test_gpu_nnsp.py tests/test_gpu_shards.py -x -q --timeout 300 --timeout-method thread ) > gpurun_out/r03/ab2_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03/ab2_pytest.log; exit 1; }
tail -1 gpurun_out/r03/ab2_pytest.log
bash profiles/r03/ab.sh $VAR "$VALS" $REPS
