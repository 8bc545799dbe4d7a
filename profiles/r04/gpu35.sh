#!/bin/bash
# round-4 final records, part 2: configs[1..3] nets, S2I acc32, the ARM_OPTIMIZED=0 build (cascade and
# VAD), strong scaling on one GPU, drop-in latency, smoke(), a torchrun world-size-1 bench
set -o pipefail
O=gpurun_out/r04/final3; mkdir -p $O
export TMPDIR=/tmp
for net in vad kws s2i; do
  timeout -k 10 300 python bench.py --net $net > $O/bench_$net.json 2> $O/bench_$net.err || { echo "bench $net failed"; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$net.json')); print('$net', round(d['value']/1e9,4), round(d['ms_per_step'],3), d['cpu_baseline']['value'])"
done
timeout -k 10 300 python bench.py --net s2i --acc32 --no-cpu-baseline > $O/bench_s2i_acc32.json 2> $O/bench_s2i_acc32.err || { echo "bench s2i acc32 failed"; exit 1; }
timeout -k 10 300 python bench.py --build portable --no-cpu-baseline > $O/bench_portable.json 2> $O/bench_portable.err || { echo "bench portable failed"; exit 1; }
timeout -k 10 300 python bench.py --build portable --net vad --no-cpu-baseline > $O/bench_portable_vad.json 2> $O/bench_portable_vad.err || { echo "bench portable vad failed"; exit 1; }
timeout -k 10 300 python bench.py --scaling strong --steps 5 --no-cpu-baseline --no-stress > $O/bench_strong_n1.json 2> $O/bench_strong.err || { echo "bench strong failed"; exit 1; }
for f in s2i_acc32 portable portable_vad strong_n1; do python -c "import json; d=json.load(open('$O/bench_$f.json')); print('$f', round(d['value']/1e9,4), round(d['ms_per_step'],3))"; done
timeout -k 10 300 python bench.py --dropin-latency > $O/dropin.json 2> $O/dropin.err || { echo "dropin failed"; exit 1; }
python -c "import json; d=json.load(open('$O/dropin.json'))['nets']; print({k:(round(v['gpu_us_per_frame_median'],1), round(v['cpu_baseline']['us_per_frame'],2)) for k,v in d.items()})"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 2 > $O/bench_torchrun_n1.json 2> $O/bench_torchrun_n1.err || { echo "torchrun bench failed"; tail -10 $O/bench_torchrun_n1.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_torchrun_n1.json')); print('torchrun n1', round(d['value']/1e9,4), round(d['ms_per_step'],3))"
echo all-ok
