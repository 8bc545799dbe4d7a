#!/bin/bash
# library streams as full-CU-mask streams (a hardware queue each?) under an RCCL process group
set -o pipefail
mkdir -p gpurun_out/r03/qm
for L in - abtest/mask/nnsp_amd/libnnsp_mi355x.so; do
  T=$( [ "$L" = "-" ] && echo base || echo mask )
  if [ "$L" = "-" ]; then unset NNSP_LIB; else export NNSP_LIB=$L; fi
  for i in 1 2; do
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline --no-stress --dist-backend nccl > gpurun_out/r03/qm/${T}_nccl$i.json 2> gpurun_out/r03/qm/err.log || { echo "$T nccl failed"; tail -5 gpurun_out/r03/qm/err.log; exit 1; }
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-stress > gpurun_out/r03/qm/${T}_plain$i.json 2> gpurun_out/r03/qm/err.log || { echo "$T plain failed"; tail -5 gpurun_out/r03/qm/err.log; exit 1; }
    python -c "import json; a=json.load(open('gpurun_out/r03/qm/${T}_nccl$i.json')); b=json.load(open('gpurun_out/r03/qm/${T}_plain$i.json')); print('$T', 'nccl', round(a['value']/1e9,4), 'plain', round(b['value']/1e9,4))"
  done
done
