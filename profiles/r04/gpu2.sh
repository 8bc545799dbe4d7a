#!/bin/bash
# NN epilogue changes: GPU parity (NN, cascade, e2e suites), then paired A/B vs the previous build
set -o pipefail
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu2.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu2.log; exit 1; }
tail -1 $O/pytest_gpu2.log
B=abtest/base/nnsp_amd/libnnsp_mi355x.so
bash profiles/r04/ab.sh NNSP_LIB "$B -" 3 && \
bash profiles/r04/ab.sh NNSP_LIB "$B -" 2 --net vad --no-stress && \
bash profiles/r04/ab.sh NNSP_LIB "$B -" 2 --net s2i --no-stress
# kernel trace of the synthetic-weight cascade (the stress line's rounds)
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_synth -o kt -- python3 bench.py --no-cpu-baseline --no-stress --weights synth --steps 3 --warmup 1 > $O/kt_synth.log 2>&1 || { echo "synth trace failed"; tail -5 $O/kt_synth.log; exit 1; }
echo trace-ok
