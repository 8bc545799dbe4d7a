#!/bin/bash
# A/B of an environment knob: each bench config alternated between the
# settings, twice.  usage: KNOB=NNSP_FE_PAIR VALS="0 1" profiles/r02/ab_env.sh OUTDIR
set -u
cd $GRAFT_REPO_ROOT
O=$1
mkdir -p $O
for rep in 1 2; do
  for cfg in "cascade:" "vad:--net vad"; do
    n=${cfg%%:*}; A=${cfg#*:}
    for v in $VALS; do
      env $KNOB=$v timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-stress $A > $O/${v}_${n}_$rep.json 2>> $O/err.log || { echo "$v $n failed"; exit 4; }
      python3 -c "import json; d=json.loads(open('$O/${v}_${n}_$rep.json').read().strip().splitlines()[-1]); print('$KNOB=$v $n $rep', round(d['value']/1e6,1), round(d['ms_per_step'],3), 'fe', round(d.get('fe_ms_per_step',0),3))"
    done
  done
done
