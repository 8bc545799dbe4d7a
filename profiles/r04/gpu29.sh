#!/bin/bash
# FE bank sums: three unconditional reads, lane 63 (no segment) as the zero slot: GPU suite, A/B against HEAD (r4f)
set -o pipefail
O=gpurun_out/r04/g29; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest29.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest29.log; exit 1; }
tail -1 $O/pytest29.log
bash profiles/r04/ab.sh NNSP_LIB "abtest/r4f/nnsp_amd/libnnsp_mi355x.so -" 4 || exit 1
echo all-ok
