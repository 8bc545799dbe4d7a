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
one base X=1
one vad X=1 -- --net vad
one kws X=1 -- --net kws
one s2i X=1 -- --net s2i
one synth X=1 -- --weights synth
one after0 NNSP_AHEAD_AFTER_ROUND=0
one prio_after0_blk2048 NNSP_NET_STREAM_PRIO=1 NNSP_AHEAD_AFTER_ROUND=0 NNSP_AHEAD_FE_BLOCKS=2048
one prio_after0_blk3072 NNSP_NET_STREAM_PRIO=1 NNSP_AHEAD_AFTER_ROUND=0 NNSP_AHEAD_FE_BLOCKS=3072
one noahead X=1 -- --no-lookahead
echo done
