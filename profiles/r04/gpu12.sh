#!/bin/bash
# LSTM tile view in registers: suite (nnsp + cascade), instruction-cache counters and per-stage
# clocks vs HEAD~ (prev) and the last commit (r4a), single-net A/B
set -o pipefail
O=gpurun_out/r04/icache; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_cascade.py tests/test_gpu_nnsp.py tests/test_gpu_benchcfg.py > $O/pytest12.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest12.log; exit 1; }
tail -1 $O/pytest12.log
for v in prev r4a cur; do
  if [ $v = cur ]; then unset NNSP_LIB; else export NNSP_LIB=abtest/$v/nnsp_amd/libnnsp_mi355x.so; fi
  for net in s2i kws; do
    timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $O/${v}_$net -o p -- python3 bench.py --net $net --no-cpu-baseline --no-stress --steps 3 --warmup 1 > $O/${v}_$net.log 2>&1 || { echo "pmc $v $net rc=$?"; tail -5 $O/${v}_$net.log; exit 1; }
    timeout -k 10 120 python profiles/recur_clocks.py $net 8192 ref > $O/clk_${v}_$net.log 2>&1 || { echo "clocks $v $net failed"; exit 1; }
    echo "$v $net: $(grep -v amdgpu.ids $O/clk_${v}_$net.log | head -6 | tr '\n' ' ')"
  done
done
unset NNSP_LIB
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/r04/icache/*/*counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0].split("<")[0]
        agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
    for k in ("recur_pipe_kernel", "proj_kernel"):
        if k in agg: print(f.split("/")[-2], k, {c: round(v) for c, v in agg[k].items()})
PY
for net in s2i kws; do
  bash profiles/r04/ab.sh NNSP_LIB "abtest/r4a/nnsp_amd/libnnsp_mi355x.so -" 2 --net $net --no-stress || exit 1
done
bash profiles/r04/ab.sh NNSP_LIB "abtest/r4a/nnsp_amd/libnnsp_mi355x.so - abtest/w3/nnsp_amd/libnnsp_mi355x.so" 2 || exit 1
bash profiles/r04/ab.sh NNSP_LIB "- abtest/w3/nnsp_amd/libnnsp_mi355x.so" 2 --net vad --no-stress || exit 1
echo all-ok
