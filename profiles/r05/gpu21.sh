#!/bin/bash
# proj's activation table from global memory (default) vs its LDS copy (PROJ_TT_LDS=1 library): GPU suite, A/B
set -o pipefail
O=gpurun_out/r05/g21; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash profiles/r05/ab2.sh projtt "NNSP_LIB=abtest/projlds/nnsp_amd/libnnsp_mi355x.so -" 4 || exit 1
bash profiles/r05/ab2.sh projtt_vad "NNSP_LIB=abtest/projlds/nnsp_amd/libnnsp_mi355x.so -" 3 --net vad || exit 1
echo all-ok
