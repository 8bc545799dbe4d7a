#!/bin/bash
# round-6 final records: full GPU suite and smoke; kernel trace + four PMC passes of the default cascade
# bench and their summary; default bench x3 on that profile; single-net configs; strong scaling on one GPU;
# torchrun world size 1; drop-in latency
set -o pipefail
O=gpurun_out/r06/final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash profiles/r05/prof.sh $O/cascade || exit 1
python3 profiles/r05/summarize.py $O/cascade cascade 32768 100 ref mix $O/pmc_cascade.json > $O/summ.log 2>&1 || { echo "summarize failed"; tail -5 $O/summ.log; exit 1; }
cat $O/summ.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --profile-json $O/pmc_cascade.json > $O/bench_cascade_$i.json 2> $O/bench_cascade_$i.err || { echo "bench $i failed"; tail -5 $O/bench_cascade_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_cascade_$i.json')); r=d['roofline']; print('cascade', round(d['value']/1e9,4), round(d['ms_per_step'],3), round(d['fe_ms_per_step'],3), round(r.get('frac'),3), r.get('valu_busy'), r.get('valu_occupancy'), d.get('cascade_synthetic_weights',{}).get('value'), d['cpu_baseline']['value'], d['cascade']['host_gap_ms'])"
done
for n in vad kws s2i; do
  timeout -k 10 300 python bench.py --net $n --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err || { echo "bench $n failed"; tail -5 $O/bench_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$n.json')); print('$n', round(d['value']/1e9,4), round(d['ms_per_step'],3))"
done
timeout -k 10 300 python bench.py --net s2i --acc32 --no-cpu-baseline > $O/bench_s2i_acc32.json 2> $O/bench_s2i_acc32.err || { echo "bench s2i acc32 failed"; exit 1; }
python -c "import json; d=json.load(open('$O/bench_s2i_acc32.json')); print('s2i acc32', round(d['value']/1e9,4), round(d['ms_per_step'],3))"
timeout -k 10 300 python bench.py --scaling strong --steps 5 --no-cpu-baseline --no-stress > $O/bench_strong_n1.json 2> $O/bench_strong.err || { echo "bench strong failed"; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline --no-stress > $O/bench_torchrun_n1.json 2> $O/bench_torchrun_n1.err || { echo "torchrun bench failed"; tail -10 $O/bench_torchrun_n1.err; exit 1; }
for f in strong_n1 torchrun_n1; do python -c "import json; d=json.load(open('$O/bench_$f.json')); print('$f', round(d['value']/1e9,4), round(d['ms_per_step'],3), d['n_gpus'])"; done
timeout -k 10 300 python bench.py --dropin-latency > $O/dropin.json 2> $O/dropin.err || { echo "dropin failed"; tail -10 $O/dropin.err; exit 1; }
python -c "import json; d=json.load(open('$O/dropin.json'))['nets']; print({k:(round(v['gpu_us_per_frame_median'],1), round(v['cpu_baseline']['us_per_frame'],2)) for k,v in d.items()})"
echo all-ok
