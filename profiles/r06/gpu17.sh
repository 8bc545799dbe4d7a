#!/bin/bash
# round 6: drop-in parity on the generic nets (LDS and memory paths)
set -o pipefail
O=gpurun_out/r06/${TAG:-g17}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_legacy.py > $O/pytest_req.log 2>&1 || { echo "pytest (required) failed"; tail -60 $O/pytest_req.log; exit 1; }
tail -14 $O/pytest_req.log
echo all-ok
