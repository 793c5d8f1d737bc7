#!/bin/bash
# Collect PMC counters for the bench workload, one rocprofv3 pass per counter group.
# usage: tools/pmc.sh <outdir> [bench args...]
set -o pipefail
OUT=$(mkdir -p "$1" && cd "$1" && pwd); shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH" \
  "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o pmc -- python "$R/bench.py" "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
python - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].split("(")[0]
        agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in agg.items():
    if "k_replay" not in k and "k_piece" not in k and "k_compact" not in k and "k_etag" not in k: continue
    print(k)
    for c, v in sorted(d.items()):
        # (per 8-KiB tile of a 4-GiB shard: 524288 tiles; SQ_*_CYCLES in quad-cycles)
        print(f"   {c:28s} mean/dispatch {sum(v)/len(v):16.1f}  per tile {sum(v)/len(v)/524288:10.1f}  (n={len(v)})")
PY
