#!/bin/bash
# final round-4 records, part 3: S2I acc32, the ARM_OPTIMIZED=0 build, strong scaling on one GPU,
# drop-in latency
set -o pipefail
O=gpurun_out/r04/final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --net s2i --acc32 --no-cpu-baseline > $O/bench_s2i_acc32.json 2> $O/bench_s2i_acc32.err || { echo "bench s2i acc32 failed"; exit 1; }
timeout -k 10 300 python bench.py --build portable > $O/bench_portable.json 2> $O/bench_portable.err || { echo "bench portable failed"; exit 1; }
timeout -k 10 300 python bench.py --build portable --net vad --no-cpu-baseline > $O/bench_portable_vad.json 2> $O/bench_portable_vad.err || { echo "bench portable vad failed"; exit 1; }
timeout -k 10 300 python bench.py --scaling strong --steps 5 --no-cpu-baseline --no-stress > $O/bench_strong_n1.json 2> $O/bench_strong.err || { echo "bench strong failed"; exit 1; }
timeout -k 10 300 python bench.py --dropin-latency > $O/dropin.json 2> $O/dropin.err || { echo "dropin failed"; exit 1; }
for f in s2i_acc32 portable portable_vad strong_n1; do python -c "import json; d=json.load(open('$O/bench_$f.json')); print('$f', round(d['value']/1e9,4), round(d['ms_per_step'],3))"; done
python -c "import json; d=json.load(open('$O/dropin.json'))['nets']; print({k:(round(v['gpu_us_per_frame_median'],1), round(v['cpu_baseline']['us_per_frame'],2)) for k,v in d.items()})"

bash profiles/r04/ab.sh NNSP_RECUR_TSEQ_VAD "- 2" 3 || exit 1
echo ab-ok
