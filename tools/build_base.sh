#!/bin/bash
# Build libfmx.so of a git revision into fmtuner-sdr_amd/libfmx_<name>.so
# (A/B runs: FMX_LIB=... python bench.py).  Usage: [KDEFS=...] tools/build_base.sh REV NAME
set -e
REV=${1:-HEAD}; NAME=${2:-base}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=/tmp/fmx_wt_$NAME
rm -rf "$WT"; git -C "$ROOT" worktree prune
git -C "$ROOT" worktree add -f "$WT" "$REV" > /dev/null 2>&1
make -C "$WT/fmtuner-sdr_amd" -j8 KDEFS="${KDEFS:-}" > /dev/null
cp "$WT/fmtuner-sdr_amd/libfmx.so" "$ROOT/fmtuner-sdr_amd/libfmx_$NAME.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "built $REV -> fmtuner-sdr_amd/libfmx_$NAME.so"
