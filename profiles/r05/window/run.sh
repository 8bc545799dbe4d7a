#!/bin/bash
# stress case (synthetic weights): fixed windows 12 / 16 (the auto rule's choice there) / 24 / 32; read synth_G
set -o pipefail
export TMPDIR=/tmp
bash profiles/r05/ab2.sh window "NNSP_CASCADE_WINDOW=16 NNSP_CASCADE_WINDOW=12 NNSP_CASCADE_WINDOW=24 NNSP_CASCADE_WINDOW=32" 4 || exit 1
echo all-ok
