#!/bin/bash
# the bench under torch.distributed.run at world size 1: RCCL vs gloo process group, more HIP hardware queues
set -o pipefail
mkdir -p gpurun_out/r03/tr
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  timeout -k 10 300 env "$@" python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline --no-stress $BARGS > gpurun_out/r03/tr/$tag.json 2> gpurun_out/r03/tr/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/r03/tr/$tag.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/r03/tr/$tag.json')); print('$tag', round(d['value']/1e9,4), round(d['ms_per_step'],3), round(d['fe_ms_per_step'],3))"
}
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-stress > gpurun_out/r03/tr/plain$i.json 2>/dev/null && python -c "import json; d=json.load(open('gpurun_out/r03/tr/plain$i.json')); print('plain', round(d['value']/1e9,4), round(d['ms_per_step'],3))"
  run nccl$i X=1 || exit 1
  BARGS="--dist-backend gloo" run gloo$i X=1 || exit 1
  run nccl_q8_$i GPU_MAX_HW_QUEUES=8 || exit 1
done
