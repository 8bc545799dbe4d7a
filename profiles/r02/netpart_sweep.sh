#!/bin/bash
# cascade bench under per-net CU partitions (NNSP_NET_CUS, nets s2i,vad,kws)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUTD:-r02np}
mkdir -p $O
i=0
for P in none 0:96,96:256,0:96 0:64,128:256,64:128 0:128,128:256,0:128 0:64,64:256,0:64 none 0:96,96:256,0:96 0:160,96:256,0:160; do
  i=$((i+1))
  if [ $P = none ]; then unset NNSP_NET_CUS; else export NNSP_NET_CUS=$P; fi
  timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-stress > $O/b$i.json 2>> $O/err.log || { echo "$P failed"; exit 4; }
  python3 -c "import json; d=json.loads(open('$O/b$i.json').read().strip().splitlines()[-1]); print('$P', round(d['value']/1e6,1), round(d['ms_per_step'],3))"
done
