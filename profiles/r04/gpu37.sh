#!/bin/bash
# later rounds' proj grid (NNSP_PROJ_LATE_BLOCKS; default: the persistent grid of the first round, most of
# whose workgroups find no tile in a short round): synthetic-weight stress line and the headline, 3 passes
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 env NNSP_PROJ_LATE_BLOCKS=128 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_cascade.py > gpurun_out/pytest37.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/pytest37.log; exit 1; }
tail -1 gpurun_out/pytest37.log
bash profiles/r04/ab.sh NNSP_PROJ_LATE_BLOCKS "- 128 256" 3 --weights synth --no-stress || exit 1
bash profiles/r04/ab.sh NNSP_PROJ_LATE_BLOCKS "- 128" 2 --no-stress || exit 1
echo all-ok
