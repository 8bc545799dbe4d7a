#!/bin/bash
# later rounds' launch order (NNSP_RN_ORDER: 0 S2I, VAD, KWS; 1 VAD, S2I, KWS; 2 KWS, S2I, VAD)
set -o pipefail
export TMPDIR=/tmp
bash profiles/r05/ab2.sh rnorder1 "- NNSP_RN_ORDER=1" 6 || exit 1
echo all-ok
