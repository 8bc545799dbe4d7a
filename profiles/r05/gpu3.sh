#!/bin/bash
# new tests + suite on the cell-state stride build; paired A/B against the round-start build;
# LDS conflict counters of the cascade's kernels
set -o pipefail
O=gpurun_out/r05/g3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cascade_state.py tests/test_gpu_benchloop.py > $O/pytest_new.log 2>&1 || { echo "new tests failed"; tail -40 $O/pytest_new.log; exit 1; }
tail -3 $O/pytest_new.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash profiles/r05/ab.sh NNSP_LIB "abtest/base/nnsp_amd/libnnsp_mi355x.so -" 3 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc -o p -- python3 bench.py --no-cpu-baseline --no-stress --steps 3 --warmup 1 > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
echo all-ok
