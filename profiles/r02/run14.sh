#!/bin/bash
# small cascade check, GPU suite, proj/fe per-wave probes, benches
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUTD:-r02p}
mkdir -p $O
NNSP_CASCADE_DEBUG=1 timeout -k 10 120 python -u profiles/r02/bisect_casc.py > $O/small.log 2>&1 || { tail -5 $O/small.log; exit 3; }
tail -1 $O/small.log
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=3 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
for n in vad kws s2i; do
  timeout -k 10 120 python3 profiles/r02/proj_waves.py $n 8192 > $O/pw_$n.log 2>&1 || exit 6
  grep -v amdgpu.ids $O/pw_$n.log | grep "events\|proj:"
done
for n in base vad kws s2i synth; do
  case $n in base) A="";; synth) A="--weights synth";; *) A="--net $n";; esac
  timeout -k 10 150 python -u bench.py --no-cpu-baseline --no-stress $A > $O/$n.json 2>> $O/err.log || { echo "$n failed"; exit 4; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', round(d['value']/1e6,1), round(d['ms_per_step'],3))"
done
