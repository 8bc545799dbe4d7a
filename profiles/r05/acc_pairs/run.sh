#!/bin/bash
# S2I acc64 vs acc32, paired (configs[3], 8 192 streams), 5 pairs
set -o pipefail
O=gpurun_out/r05/acc; mkdir -p $O
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --net s2i --no-cpu-baseline > $O/acc64_$i.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
  timeout -k 10 300 python bench.py --net s2i --acc32 --no-cpu-baseline > $O/acc32_$i.json 2> $O/err.log || { tail -5 $O/err.log; exit 1; }
done
python - <<'PY'
import json
for a in ("acc64", "acc32"):
    print(a, [round(json.load(open(f"gpurun_out/r05/acc/{a}_{i}.json"))["value"] / 1e9, 4) for i in range(1, 6)])
PY
echo all-ok
