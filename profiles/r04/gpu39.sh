#!/bin/bash
# shared front end grid, re-swept on the final FE (NNSP_FE_GENS generations of 1 536 workgroups;
# default 8 = 12 288 workgroups): cascade A/B, 3 passes
set -o pipefail
export TMPDIR=/tmp
bash profiles/r04/ab.sh NNSP_FE_GENS "${GS:-- 6 10 12}" 3 || exit 1
echo all-ok
