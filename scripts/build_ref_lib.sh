#!/bin/bash
# Build libxfgstark.so from a git revision (default HEAD) into build/libxfgstark_<rev>.so for same-box
# A/B runs against the working tree (scripts/lib_ab.sh: A=... B=...)
set -e
REV=${1:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" worktree add -q --detach "$TMP" "$REV"
make -s -j8 -C "$TMP/xfg-stark_amd"
mkdir -p "$ROOT/build"
cp "$TMP/xfg-stark_amd/libxfgstark.so" "$ROOT/build/libxfgstark_$(git -C "$ROOT" rev-parse --short "$REV").so"
git -C "$ROOT" worktree remove --force "$TMP"
ls -la "$ROOT/build/"
