#!/bin/bash
# synthetic-weight stress line: recur tiles per workgroup at W = 16 (8 NN steps; default tseq 4) against
# 2 and 3 (NNSP_RECUR_TSEQ forces every round), 3 passes
set -o pipefail
export TMPDIR=/tmp
bash profiles/r04/ab.sh NNSP_RECUR_TSEQ "- 2 3" 3 --weights synth --no-stress || exit 1
echo all-ok
