#!/bin/bash
# recur per-stage clocks (reference nets) for each library variant, then ab.sh
set -u
cd $GRAFT_REPO_ROOT
for v in $VARIANTS; do
  for n in kws s2i; do
    echo "== $v $n"; NNSP_LIB=abtest/$v/nnsp_amd/libnnsp_mi355x.so timeout -k 10 120 python -u profiles/recur_clocks.py $n 8192 ref || exit 4
  done
done
bash profiles/r02/ab.sh
