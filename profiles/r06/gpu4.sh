#!/bin/bash
# round 6: fused VAD prefix (NNSP_FUSE_PREFIX): GPU suite with it on, the bench loop requiring it, paired A/B
set -o pipefail
O=gpurun_out/r06/g4; mkdir -p $O
export TMPDIR=/tmp
NNSP_FUSE_PREFIX=2 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_benchloop.py tests/test_gpu_benchcfg.py > $O/pytest_req.log 2>&1 || { echo "pytest (required) failed"; tail -40 $O/pytest_req.log; exit 1; }
tail -1 $O/pytest_req.log
NNSP_FUSE_PREFIX=1 timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash profiles/r06/ab.sh NNSP_FUSE_PREFIX "0 1" 3 || exit 1
echo all-ok
