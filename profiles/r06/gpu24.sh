#!/bin/bash
# round 6: VAD proj at <= 80 VGPRs (PROJ_MINW_SMALL=6: three 8-wave workgroups per CU instead of two) -- paired A/B,
# cascade and single-net VAD; kernel trace of both for proj's duration
set -o pipefail
O=gpurun_out/r06/${TAG:-g24}; mkdir -p $O
export TMPDIR=/tmp
NNSP_LIB=abtest/pw6/nnsp_amd/libnnsp_mi355x.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_benchloop.py tests/test_gpu_refnets.py > $O/pytest_req.log 2>&1 || { echo "pytest (required) failed"; tail -40 $O/pytest_req.log; exit 1; }
tail -1 $O/pytest_req.log
rm -rf gpurun_out/r06/ab_NNSP_LIB
bash profiles/r06/ab.sh NNSP_LIB "- abtest/pw6/nnsp_amd/libnnsp_mi355x.so" 4 || exit 1
mv gpurun_out/r06/ab_NNSP_LIB $O/ab_cascade
bash profiles/r06/ab.sh NNSP_LIB "- abtest/pw6/nnsp_amd/libnnsp_mi355x.so" 3 --net vad || exit 1
mv gpurun_out/r06/ab_NNSP_LIB $O/ab_vad
for v in base pw6; do
  if [ $v = pw6 ]; then export NNSP_LIB=abtest/pw6/nnsp_amd/libnnsp_mi355x.so; else unset NNSP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o kt -- python3 bench.py --no-cpu-baseline --no-stress --steps 3 --warmup 1 > $O/kt_$v.log 2>&1 || { echo "kt $v failed"; tail -5 $O/kt_$v.log; exit 1; }
  grep -h "proj_kernel\|recur_pipe" $O/kt_$v/kt_kernel_stats.csv | cut -c1-200 | sed "s/^/$v: /" | head -12
done
unset NNSP_LIB
echo all-ok
