#!/bin/bash
# guided shared front end schedule: tail waves (twelfths of the grid) and share divisor (NNSP_FE_GUIDE)
set -o pipefail
export TMPDIR=/tmp
bash profiles/r05/ab2.sh guide "NNSP_FE_GUIDE=4,4 NNSP_FE_GUIDE=6,6 NNSP_FE_GUIDE=3,3 NNSP_FE_GUIDE=4,6 NNSP_FE_GUIDE=8,8" 3 || exit 1
echo all-ok
