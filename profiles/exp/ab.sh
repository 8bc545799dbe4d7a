# A/B of library builds in profiles/exp/ab/*.so on one bench workload (alternating, 2 rounds)
#   usage: profiles/exp/ab.sh NET
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/ab
for i in 1 2; do for L in profiles/exp/ab/*.so; do
  n=$(basename $L .so)
  NNSP_LIB=$PWD/$L timeout -k 10 200 python3 bench.py --net $1 --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || { echo "$n failed"; tail -5 gpurun_out/ab/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab/$n.json')); print('$n', round(d['value']/1e6,1), {k: round(v,4) for k,v in d['kernels_ms_per_step'].items()})"
done; done
