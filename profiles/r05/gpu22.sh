#!/bin/bash
# new cascade tests (schedule knobs, tiny grids); front-end generations on the guided schedule
set -o pipefail
O=gpurun_out/r05/g22; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cascade.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash profiles/r05/ab2.sh fegens "- NNSP_FE_GENS=4 NNSP_FE_GENS=5 NNSP_FE_GENS=8" 3 || exit 1
echo all-ok
