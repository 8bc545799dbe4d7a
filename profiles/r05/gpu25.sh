#!/bin/bash
# round-0 launch order: S2I first (6: S2I, VAD, KWS; 7: S2I, KWS, VAD), nothing waits
set -o pipefail
export TMPDIR=/tmp
bash profiles/r05/ab2.sh r0order2 "- NNSP_R0_ORDER=6 NNSP_R0_ORDER=7" 4 || exit 1
echo all-ok
