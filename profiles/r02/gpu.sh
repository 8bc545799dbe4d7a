#!/bin/bash
# gpurun with a bounded retry of infrastructure-side transient failures only
# (status "transient": nothing ran, nothing charged); any other outcome returns.
# usage: profiles/r02/gpu.sh TIMEOUT 'command'
T=$1; shift
for i in 1 2 3 4 5; do
  /usr/local/graft/bin/gpurun --timeout $T -- "$@"
  rc=$?
  st=$(python3 -c "import json; print(json.load(open('/root/repo/gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
  [ "$st" = "transient" ] || exit $rc
  echo "[gpu.sh] transient ($i), waiting 60 s"; sleep 60
done
exit $rc
