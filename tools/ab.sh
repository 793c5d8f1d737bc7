#!/bin/bash
# A/B timing of k_replay builds (tools/ablate.py cfg2: masks under lib/ablate, names under
# lib/variants) and, optionally, their per-tile PMC counters (tools/pmc_variants.sh).
#   usage: tools/ab.sh <tag> "<timed builds>" "<pmc builds>" [cfg]
set -o pipefail
T=$1; A=$2; P=$3; CFG=${4:-cfg2}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/gpurun_out/$T"
for m in $A; do
  timeout -k 10 120 python -u "$R/tools/ablate.py" $CFG 0 $m >> "$R/gpurun_out/$T/ab.txt" 2>&1 || { echo "build $m failed"; tail -5 "$R/gpurun_out/$T/ab.txt"; exit 1; }
done
cat "$R/gpurun_out/$T/ab.txt"
if [ -n "$P" ]; then
  bash "$R/tools/pmc_variants.sh" "$R/gpurun_out/$T/pmc" $P > "$R/gpurun_out/$T/pmc.txt" 2>&1 || { echo "pmc failed"; tail -20 "$R/gpurun_out/$T/pmc.txt"; exit 1; }
  cat "$R/gpurun_out/$T/pmc.txt"
fi
