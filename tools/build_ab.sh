#!/bin/bash
# Build libkvreplay.so variants for A/B timing into lib/ab/ (tools/ablate.py <cfg> 0 <name>):
#   tools/build_ab.sh <name> <git-rev|WORK> [-Dflags...]
# WORK builds the working tree's sources; a git revision builds that commit's csrc + include.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; REV=$2; shift 2
OUT=$R/mini-kvstore-v2_amd/lib/ab
mkdir -p "$OUT"
if [ "$REV" = WORK ]; then
  SRC=$R
else
  SRC=$(mktemp -d)
  (cd "$R" && git archive "$REV" mini-kvstore-v2_amd/csrc include) | tar -x -C "$SRC"
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result "$@" \
  -o "$OUT/libkvreplay_$NAME.so" "$SRC/mini-kvstore-v2_amd/csrc/kvr_api.hip"
echo "built $OUT/libkvreplay_$NAME.so"
