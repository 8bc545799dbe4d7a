#!/bin/bash
# A/B of library variants under abtest/<name>/nnsp_amd (development): each
# bench config alternated between the variants, twice
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUTD:-ab}
mkdir -p $O
for rep in 1 2; do
  for cfg in "cascade:" "vad:--net vad"; do
    n=${cfg%%:*}; A=${cfg#*:}
    for v in $VARIANTS; do
      NNSP_LIB=abtest/$v/nnsp_amd/libnnsp_mi355x.so timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-stress $A > $O/${v}_${n}_$rep.json 2>> $O/err.log || { echo "$v $n failed"; exit 4; }
      python3 -c "import json; d=json.loads(open('$O/${v}_${n}_$rep.json').read().strip().splitlines()[-1]); print('$v $n $rep', round(d['value']/1e6,1), round(d['ms_per_step'],3), 'fe', round(d.get('fe_ms_per_step',0),3))"
    done
  done
done
