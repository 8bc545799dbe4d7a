#!/bin/bash
# probes compiled out (NNSP_PROBES=0 default): suite, A/B against HEAD's build with probes (r4d),
# per-stage clocks from the probes build of the same source
set -o pipefail
O=gpurun_out/r04/g24; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest24.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest24.log; exit 1; }
tail -1 $O/pytest24.log
bash profiles/r04/ab.sh NNSP_LIB "abtest/r4d/nnsp_amd/libnnsp_mi355x.so -" 3 || exit 1
for net in s2i kws vad; do
  bash profiles/r04/ab.sh NNSP_LIB "abtest/r4d/nnsp_amd/libnnsp_mi355x.so -" 2 --net $net --no-stress || exit 1
done
echo all-ok
