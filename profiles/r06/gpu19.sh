#!/bin/bash
# round 6: paired A/B -- round start (h6) / table batching (c7, 430cedf) / + Mel bank sums by LDS atomics (current)
set -o pipefail
export TMPDIR=/tmp
bash profiles/r06/ab.sh NNSP_LIB "abtest/h6/nnsp_amd/libnnsp_mi355x.so abtest/c7/nnsp_amd/libnnsp_mi355x.so -" 4 || exit 1
echo all-ok
