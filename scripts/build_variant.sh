#!/bin/bash
# CPU container: build the working tree's libxfgstark.so with extra compile flags (e.g. an A/B macro)
# into OUT: scripts/build_variant.sh build/libxfgstark_x.so -DXFG_PAIR_STORES=0
set -e
OUT=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/xfg_var.XXXX)
mkdir -p $T/xfg-stark_amd $T/include
cp -r "$ROOT/xfg-stark_amd/csrc" "$ROOT/xfg-stark_amd/Makefile" $T/xfg-stark_amd/
cp "$ROOT/include/"*.h $T/include/
make -s -j8 -C $T/xfg-stark_amd CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $*"
mkdir -p "$(dirname "$ROOT/$OUT")"
cp $T/xfg-stark_amd/libxfgstark.so "$ROOT/$OUT"
rm -rf $T
echo "built $OUT ($*)"
