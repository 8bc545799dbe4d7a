#!/bin/bash
# round 6: fused prefix (two waves) parity + clocks + A/B; drop-in phase probes
set -o pipefail
O=gpurun_out/r06/g10; mkdir -p $O
export TMPDIR=/tmp


TAG=g10 bash profiles/r06/gpu7.sh || exit 1
echo all-ok
