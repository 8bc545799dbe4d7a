#!/bin/bash
# Build the library of another git revision into abtest/<name>/ for paired
# A/B runs on one GPU box (NNSP_LIB=abtest/<name>/nnsp_amd/libnnsp_mi355x.so).
# usage: tools/build_rev.sh REV NAME
set -e
REV=$1; NAME=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
DST=$ROOT/abtest/$NAME
rm -rf "$DST"
mkdir -p "$DST"
git -C "$ROOT" archive "$REV" nnsp_amd include | tar -x -C "$DST"
cd "$DST"
python3 -c "import sys; sys.path.insert(0, '.'); from nnsp_amd import tables; tables.write_header()"
make -C nnsp_amd -j8 > /dev/null
rm -rf nnsp_amd/build
echo "$DST/nnsp_amd/libnnsp_mi355x.so"
