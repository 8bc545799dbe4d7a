#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u profiles/r03/wg_timeline.py 32768 gpurun_out/r03/wg_records.npz > gpurun_out/r03/wg_timeline.txt 2>&1 || { tail -20 gpurun_out/r03/wg_timeline.txt; exit 1; }
head -12 gpurun_out/r03/wg_timeline.txt
