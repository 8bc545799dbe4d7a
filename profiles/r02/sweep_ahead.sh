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
one free16s NNSP_FE_FREE_CUS=16
one free32s NNSP_FE_FREE_CUS=32
one free64s NNSP_FE_FREE_CUS=64
one free32t NNSP_FE_FREE_CUS=32 NNSP_FE_FREE_SPREAD=0
one free32s_prio NNSP_FE_FREE_CUS=32 NNSP_NET_STREAM_PRIO=1
one free32s_after0 NNSP_FE_FREE_CUS=32 NNSP_AHEAD_AFTER_ROUND=0
one free64s_after0 NNSP_FE_FREE_CUS=64 NNSP_AHEAD_AFTER_ROUND=0
one free32s_after2 NNSP_FE_FREE_CUS=32 NNSP_AHEAD_AFTER_ROUND=2
one after2 NNSP_AHEAD_AFTER_ROUND=2
one after3 NNSP_AHEAD_AFTER_ROUND=3
echo done
