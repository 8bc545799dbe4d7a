#!/bin/bash
# Round-1 profile: kernel trace + stats and the two HBM counter passes for one
# bench workload.  usage: profiles/collect_r01.sh WORKLOAD [extra bench args]
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
W=$1; shift
D=gpurun_out/prof_$W
mkdir -p $D
S=$( [ "$W" = cascade ] && echo 32768 || echo 8192 )
B="python3 bench.py --net $W --no-cpu-baseline --steps 3 --warmup 1 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/kt -o kt -- $B > $D/kt.log 2>&1 || { echo "kt failed"; tail -5 $D/kt.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o fetch -- $B > $D/fetch.log 2>&1 || { echo "fetch failed"; tail -5 $D/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o write -- $B > $D/write.log 2>&1 || { echo "write failed"; tail -5 $D/write.log; exit 1; }
python3 profiles/pmc_summary.py $D $W $S 100 $D/summary.json
