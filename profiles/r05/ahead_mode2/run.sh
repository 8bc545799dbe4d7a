#!/bin/bash
# look-ahead front end start: after round 1's proj (mode 1, default) vs after round 1's end (mode 2), final build
set -o pipefail
export TMPDIR=/tmp
bash profiles/r05/ab2.sh amode "- NNSP_AHEAD_MODE=2" 5 || exit 1
echo all-ok
