#!/bin/bash
# plain launch vs torch.distributed.run at world size 1, alternating (the driver's SCALE runs use the latter)
set -o pipefail
O=gpurun_out/r05/g12; mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-stress > $O/plain_$i.json 2> $O/plain.err || { echo "plain failed"; exit 1; }
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2951$i bench.py --gpus 1 --no-cpu-baseline --no-stress > $O/trun_$i.json 2> $O/trun.err || { echo "torchrun failed"; tail -5 $O/trun.err; exit 1; }
done
python - <<'PY'
import json
for k in ("plain", "trun"):
    v = [json.load(open(f"gpurun_out/r05/g12/{k}_{i}.json")) for i in (1, 2, 3)]
    print(k, [round(d["value"] / 1e9, 4) for d in v], [round(d["cascade"]["host_gap_ms"], 4) for d in v],
          [round(d["fe_ms_per_step"], 3) for d in v])
PY
echo all-ok
