#!/bin/bash
# round-0 order 6 default: cascade suites; casc_begin on S2I's / KWS's stream instead of VAD's
set -o pipefail
O=gpurun_out/r05/g27; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cascade.py tests/test_gpu_benchloop.py tests/test_gpu_cascade_state.py tests/test_gpu_benchcfg.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash profiles/r05/ab2.sh beginnet "- NNSP_BEGIN_NET=0 NNSP_BEGIN_NET=2" 4 || exit 1
echo all-ok
