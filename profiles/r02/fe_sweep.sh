set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02fb; mkdir -p $O
for B in ${BLIST:-6144 1536 3072}; do
  echo "== blocks $B"
  NNSP_FE_BLOCKS=$B timeout -k 10 120 python3 profiles/r02/fe_waves.py vad 32768 2>&1 | grep -v amdgpu.ids || exit 3
  for n in vad base; do
    case $n in base) A="";; *) A="--net $n";; esac
    NNSP_FE_BLOCKS=$B timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-stress $A > $O/$n$B.json 2>> $O/err.log || { echo "$n failed"; exit 4; }
    python3 -c "import json; d=json.loads(open('$O/$n$B.json').read().strip().splitlines()[-1]); print('$n', round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d.get('fe_ms_per_step',0),3))"
  done
done
