#!/bin/bash
# shared front end at seven waves per SIMD (seven-wave workgroups, four per CU): suite, A/B against
# HEAD's build (r4e)
set -o pipefail
O=gpurun_out/r04/g25; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_cascade.py tests/test_gpu_benchcfg.py tests/test_gpu_bigshard.py > $O/pytest25.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest25.log; exit 1; }
tail -1 $O/pytest25.log
bash profiles/r04/ab.sh NNSP_LIB "abtest/r4e/nnsp_amd/libnnsp_mi355x.so -" 3 || exit 1
echo all-ok
