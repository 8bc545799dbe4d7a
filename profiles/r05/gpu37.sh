#!/bin/bash
# look-ahead front end after round last_rounds - k (NNSP_AHEAD_LATE=k) when the last chunk needed > 4 rounds: stress
set -o pipefail
export TMPDIR=/tmp
bash profiles/r05/ab2.sh aheadlate3 "- NNSP_AHEAD_LATE=3 NNSP_AHEAD_LATE=5 NNSP_AHEAD_LATE=7" 3 --weights synth --no-stress || exit 1
echo all-ok
