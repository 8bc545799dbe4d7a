#!/bin/bash
# cold front end grid cap (NNSP_COLD_FE_BLOCKS; default 2048 workgroups for the device-sized cold lists,
# most of which exit at once): cascade A/B (reference weights + the synthetic stress line), 3 passes
set -o pipefail
export TMPDIR=/tmp
bash profiles/r04/ab.sh NNSP_COLD_FE_BLOCKS "- 256 512 1024" 3 || exit 1
echo all-ok
