#!/bin/bash
# single-net bench lines (BASELINE configs[1..3]: VAD, KWS, S2I at 8192 streams;
# S2I with both accumulators) plus a kernel-trace --stats profile of each, and
# a kernel trace + stats of the default cascade line
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/r03/lines
mkdir -p $D
run() {   # tag, bench args...
  local tag=$1; shift
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 "$@" > $D/$tag.json 2> $D/$tag.err || { echo "$tag failed"; tail -5 $D/$tag.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_$tag -o $tag -- python3 bench.py --no-cpu-baseline --no-stress --steps 10 --warmup 2 "$@" > $D/prof_$tag.log 2>&1 || { echo "prof $tag failed"; tail -5 $D/prof_$tag.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$D/$tag.json')); print('$tag', round(d['value']/1e6,1), 'M frames/s', round(d['ms_per_step'],3), 'ms/step', 'cpu', round(d.get('cpu_baseline',{}).get('value',0)/1e6,3))"
}
run vad --net vad
run kws --net kws
run s2i64 --net s2i
run s2i32 --net s2i --acc32
run vad32 --net vad --acc32
run kws32 --net kws --acc32
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof_cascade -o cascade -- python3 bench.py --no-cpu-baseline --no-stress --steps 6 --warmup 2 > $D/prof_cascade.log 2>&1 || { echo "prof cascade failed"; tail -5 $D/prof_cascade.log; exit 1; }
echo lines-ok
