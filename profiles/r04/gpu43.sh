#!/bin/bash
# synthetic-weight stress line, recur tiles per workgroup per net: VAD kept at 4 (NNSP_RECUR_TSEQ_VAD),
# S2I and KWS at 4 (default) / 2 / 3, 3 passes
set -o pipefail
export TMPDIR=/tmp
export NNSP_RECUR_TSEQ_VAD=4
bash profiles/r04/ab.sh NNSP_RECUR_TSEQ "- 2 3" 3 --weights synth --no-stress || exit 1
echo all-ok
