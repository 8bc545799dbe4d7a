#!/bin/bash
# round 6: front end -- Mel bank sums by LDS atomics (one read per bank in the tail); full GPU suite (required),
# headline A/B against the round's start (abtest/h6), PMC profile of the default bench
set -o pipefail
O=gpurun_out/r06/${TAG:-g18}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/pytest_all.log 2>&1 || { echo "pytest (required) failed"; tail -40 $O/pytest_all.log; exit 1; }
tail -1 $O/pytest_all.log
bash profiles/r06/ab.sh NNSP_LIB "abtest/h6/nnsp_amd/libnnsp_mi355x.so -" 3 || exit 1
bash profiles/r05/prof.sh $O/prof || exit 1
python3 profiles/r05/summarize.py $O/prof cascade 32768 100 ref mix $O/pmc_cascade.json > $O/summ.log 2>&1 || { echo "summarize failed"; tail -5 $O/summ.log; exit 1; }
grep -i "fe_kernel\|valu_per_frame\|VALU" $O/summ.log | head -12
echo all-ok
