#!/bin/bash
# on the guided front end: high-priority net streams (all three) and early return, alone and together
set -o pipefail
export TMPDIR=/tmp
bash profiles/r05/ab2.sh prio_early "- NNSP_NET_PRIO=7 NNSP_EARLY_RETURN=1 NNSP_NET_PRIO=7+NNSP_EARLY_RETURN=1" 4 || exit 1
echo all-ok
