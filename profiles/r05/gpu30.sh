#!/bin/bash
# cold front end grid cap for device-sized lists (NNSP_COLD_FE_BLOCKS; default 2 048)
set -o pipefail
export TMPDIR=/tmp
bash profiles/r05/ab2.sh coldfe "- NNSP_COLD_FE_BLOCKS=256 NNSP_COLD_FE_BLOCKS=512 NNSP_COLD_FE_BLOCKS=128" 4 || exit 1
echo all-ok
