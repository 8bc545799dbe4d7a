#!/bin/bash
# FE tail: log10's shift as one 64-bit shift, the mean folded into the normalisation MAD (nc table),
# one branch for the three nets' normalisations: GPU suite (FE + cascade + batch), A/B against HEAD (r4e)
set -o pipefail
O=gpurun_out/r04/g28; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest28.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest28.log; exit 1; }
tail -1 $O/pytest28.log
bash profiles/r04/ab.sh NNSP_LIB "abtest/r4e/nnsp_amd/libnnsp_mi355x.so -" 4 || exit 1
echo all-ok
