#!/bin/bash
# round-4 records on the probes-off build, part 2: configs[1..3] nets, S2I acc32, the ARM_OPTIMIZED=0
# build, strong scaling on one GPU; then A/B of the FE transposes through LDS (FE_XPOSE_LDS 1 / 3)
set -o pipefail
O=gpurun_out/r04/final2; mkdir -p $O
export TMPDIR=/tmp
for net in vad kws s2i; do
  timeout -k 10 300 python bench.py --net $net > $O/bench_$net.json 2> $O/bench_$net.err || { echo "bench $net failed"; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$net.json')); print('$net', round(d['value']/1e9,4), round(d['ms_per_step'],3), d['cpu_baseline']['value'])"
done
timeout -k 10 300 python bench.py --net s2i --acc32 --no-cpu-baseline > $O/bench_s2i_acc32.json 2> $O/bench_s2i_acc32.err || { echo "bench s2i acc32 failed"; exit 1; }
timeout -k 10 300 python bench.py --build portable --no-cpu-baseline > $O/bench_portable.json 2> $O/bench_portable.err || { echo "bench portable failed"; exit 1; }
timeout -k 10 300 python bench.py --scaling strong --steps 5 --no-cpu-baseline --no-stress > $O/bench_strong_n1.json 2> $O/bench_strong.err || { echo "bench strong failed"; exit 1; }
for f in s2i_acc32 portable strong_n1; do python -c "import json; d=json.load(open('$O/bench_$f.json')); print('$f', round(d['value']/1e9,4), round(d['ms_per_step'],3))"; done
bash profiles/r04/ab.sh NNSP_LIB "abtest/r4e/nnsp_amd/libnnsp_mi355x.so abtest/xl1/nnsp_amd/libnnsp_mi355x.so abtest/xl3/nnsp_amd/libnnsp_mi355x.so" 3 || exit 1
echo all-ok
