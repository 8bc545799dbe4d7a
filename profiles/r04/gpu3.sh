#!/bin/bash
# GPU suite on the 11-MAC Mel build; reference-weight cascade kernel trace (round-0 timeline);
# synthetic-weight window sweep; drop-in single-stream latency; S2I acc32 vs acc64 on one box
set -o pipefail
O=gpurun_out/r04; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu3.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu3.log; exit 1; }
tail -1 $O/pytest_gpu3.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_ref -o kt -- python3 bench.py --no-cpu-baseline --no-stress --steps 3 --warmup 1 > $O/kt_ref.log 2>&1 || { echo "ref trace failed"; tail -5 $O/kt_ref.log; exit 1; }
echo trace-ok
for W in 8 12 16 24 32 0; do
  NNSP_CASCADE_WINDOW=$W timeout -k 10 200 python bench.py --no-cpu-baseline --no-stress --weights synth --steps 5 > $O/synth_w$W.json 2> $O/synth_err.log || { echo "synth W=$W failed"; tail -5 $O/synth_err.log; exit 1; }
  python -c "import json; d=json.load(open('$O/synth_w$W.json')); print('W=$W', round(d['value']/1e9,4), 'G rounds', d['cascade']['rounds_per_step'], 'spec', round(d['cascade']['speculation_overhead'],3))"
done
timeout -k 10 300 python bench.py --dropin-latency > $O/dropin.json 2> $O/dropin.err || { echo "dropin failed"; tail -10 $O/dropin.err; exit 1; }
cat $O/dropin.json
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --net s2i > $O/s2i64_$i.json 2>/dev/null && timeout -k 10 200 python bench.py --no-cpu-baseline --net s2i --acc32 > $O/s2i32_$i.json 2>/dev/null || { echo "s2i ab failed"; exit 1; }
done
python -c "
import json
for a in ('64','32'):
    print('s2i acc'+a, [round(json.load(open('$O/s2i%s_%d.json'%(a,i)))['value']/1e9,4) for i in (1,2)], [round(json.load(open('$O/s2i%s_%d.json'%(a,i)))['nn_ms_per_step'],4) for i in (1,2)])
"
