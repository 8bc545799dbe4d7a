#!/bin/bash
# new tests (timed-pipeline parity, cascade state export/import), then the whole GPU suite
set -o pipefail
O=gpurun_out/r05/g2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cascade_state.py tests/test_gpu_benchloop.py > $O/pytest_new.log 2>&1 || { echo "new tests failed"; tail -40 $O/pytest_new.log; exit 1; }
tail -3 $O/pytest_new.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
echo all-ok
