#!/bin/bash
# round-end checks on the final build: smoke(), a torchrun world-size-1 bench (the driver's N>1 launch
# path), the default bench once more
set -o pipefail
O=gpurun_out/r04/final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 10 --warmup 2 > $O/bench_torchrun_n1.json 2> $O/bench_torchrun_n1.err || { echo "torchrun bench failed"; tail -10 $O/bench_torchrun_n1.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_torchrun_n1.json')); print('torchrun n1', round(d['value']/1e9,4), round(d['ms_per_step'],3))"
echo all-ok
