#!/bin/bash
# round-0 launch order 6 (S2I, VAD, KWS) vs the default (VAD, S2I, KWS), 6 pairs
set -o pipefail
export TMPDIR=/tmp
bash profiles/r05/ab2.sh r0order6 "- NNSP_R0_ORDER=6" 6 || exit 1
echo all-ok
