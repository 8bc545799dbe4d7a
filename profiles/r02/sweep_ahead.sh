#!/bin/bash
# look-ahead front-end scheduling sweep on the default bench (ref cascade)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUTD:-r02s}
mkdir -p $O
one() {  # name env... [-- bench args]
  n=$1; shift
  E=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do E+=("$1"); shift; done; [ $# -gt 0 ] && shift
  env "${E[@]}" timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-stress --steps 10 --warmup 2 "$@" > $O/$n.json 2>> $O/err.log || { echo "$n failed"; exit 4; }
  python3 -c "import json,sys; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', round(d['value']/1e6,1), round(d['ms_per_step'],3))"
}
one v0 X=1
one n0 NNSP_VAD_LAST=0
one v1 X=1
one n1 NNSP_VAD_LAST=0
one v2 X=1
one n2 NNSP_VAD_LAST=0
one vs X=1 -- --weights synth
one ns NNSP_VAD_LAST=0 -- --weights synth
one vs2 X=1 -- --weights synth
one ns2 NNSP_VAD_LAST=0 -- --weights synth
echo done
