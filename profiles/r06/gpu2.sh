#!/bin/bash
# round 6: reference-object interop tests, cascade state and legacy suites
set -o pipefail
O=gpurun_out/r06/g2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cascade_ref.py tests/test_gpu_cascade_state.py tests/test_gpu_legacy.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo all-ok
