#!/bin/bash
# the look-ahead front end waiting for fewer round-1 proj events (NNSP_AHEAD_WAIT bitmask by NNSP_ID; 7 = all)
set -o pipefail
export TMPDIR=/tmp
bash profiles/r05/ab2.sh aheadwait "- NNSP_AHEAD_WAIT=1 NNSP_AHEAD_WAIT=2 NNSP_AHEAD_WAIT=0" 4 || exit 1
echo all-ok
