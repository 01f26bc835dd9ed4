#!/bin/bash
# CPU container: build libxfgstark.so of git revision REV (default HEAD) into OUT (default
# build/libxfgstark_b.so) from a temporary worktree -- the B side of scripts/lib_ab.sh (XFG_LIB)
set -e
REV=${1:-HEAD}
OUT=${2:-build/libxfgstark_b.so}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/xfg_rev.XXXX)
git -C "$ROOT" worktree add -q --detach "$WT" "$REV"
make -s -j8 -C "$WT/xfg-stark_amd"
mkdir -p "$(dirname "$ROOT/$OUT")"
cp "$WT/xfg-stark_amd/libxfgstark.so" "$ROOT/$OUT"
git -C "$ROOT" worktree remove --force "$WT"
echo "built $REV -> $OUT"
