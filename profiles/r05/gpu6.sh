#!/bin/bash
# affine activation tables (act_q15) in the NN kernels: suite, A/B vs round start; then round-0 stream priority
set -o pipefail
O=gpurun_out/r05/g6; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash profiles/r05/ab.sh NNSP_LIB "abtest/base/nnsp_amd/libnnsp_mi355x.so -" 3 || exit 1
bash profiles/r05/ab.sh NNSP_NET_PRIO "- 5 7" 2 || exit 1
export NNSP_NET_PRIO=5
bash profiles/r05/ab.sh NNSP_R0_ORDER "3 4" 2 || exit 1
echo all-ok
