#!/bin/bash
# Build the working tree's library with extra compile flags into abtest/<name>/
# for paired A/B runs (NNSP_LIB=abtest/<name>/nnsp_amd/libnnsp_mi355x.so).
# usage: tools/build_flags.sh NAME "-DFOO=1 -DBAR=2"
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
DST=$ROOT/abtest/$NAME
rm -rf "$DST"
mkdir -p "$DST/nnsp_amd"
cp -r "$ROOT/include" "$DST/"
(cd "$ROOT/nnsp_amd" && tar -c --exclude=build --exclude='*.so' csrc Makefile) | tar -x -C "$DST/nnsp_amd"
make -C "$DST/nnsp_amd" -j8 EXTRA_HIPFLAGS="$FLAGS" > /dev/null
rm -rf "$DST/nnsp_amd/build"
echo "$DST/nnsp_amd/libnnsp_mi355x.so"
