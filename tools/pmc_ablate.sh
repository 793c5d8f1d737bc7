#!/bin/bash
# Instruction counts of k_replay per ablation variant (tools/ablate.py), one rocprofv3 --pmc
# pass per variant: shows which phase the VALU / SALU / LDS instructions per tile come from.
#   usage: tools/pmc_ablate.sh <outdir> [variants...]
set -o pipefail
OUT=$(mkdir -p "$1" && cd "$1" && pwd); shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
for m in ${*:-0 1 2 3 8 16 32}; do
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_VMEM \
    --output-format csv -d "$OUT/a$m" -o pmc -- python "$R/tools/ablate.py" cfg2 0 $m > "$OUT/a$m.log" 2>&1 || { echo "variant $m failed"; tail -5 "$OUT/a$m.log"; exit 1; }
done
python - "$OUT" <<'PY'
import csv, glob, sys, collections, os
out = sys.argv[1]
for d in sorted(glob.glob(out + "/a*/")):
    agg = collections.defaultdict(list)
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if "k_replay" in row["Kernel_Name"]:
                agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
    tiles = 524288
    print(os.path.basename(d.rstrip("/")), "  ".join(f"{c}/tile={sum(v)/len(v)/tiles:.0f}" for c, v in sorted(agg.items())))
PY
