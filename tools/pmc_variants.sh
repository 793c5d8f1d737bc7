#!/bin/bash
# Per-tile PMC counters of k_piece and k_replay's first pass for ablation variants / A/B builds (tools/ablate.py
# $PCFG, default cfg2): three rocprofv3 --pmc passes per variant (counter groups within the gfx950
# per-pass limits).
#   usage: [PCFG=cfg4] tools/pmc_variants.sh <outdir> [masks or build names...]
set -o pipefail
OUT=$(mkdir -p "$1" && cd "$1" && pwd); shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
G1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAVES"
G2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
G3="SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for m in ${*:-0 3 64}; do
  g=0
  for grp in "$G1" "$G2" "$G3"; do
    g=$((g+1))
    timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/a$m/g$g" -o pmc -- python "$R/tools/ablate.py" ${PCFG:-cfg2} 0 $m \
      > "$OUT/a$m.g$g.log" 2>&1 || { echo "variant $m group $g failed"; tail -5 "$OUT/a$m.g$g.log"; exit 1; }
  done
done
python - "$OUT" <<'PY'
import csv, glob, sys, collections, os
out = sys.argv[1]
tiles = 524288
for d in sorted(glob.glob(out + "/a*/")):
    agg = collections.defaultdict(list)
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for kern in ("k_piece", "k_replay"):
            rows = [r for r in csv.DictReader(open(f)) if kern in r["Kernel_Name"]]
            if not rows: continue
            big = max(int(r["Grid_Size"]) for r in rows)
            for r in rows:
                if int(r["Grid_Size"]) == big:
                    agg[(kern, r["Counter_Name"])].append(float(r["Counter_Value"]))
    print(os.path.basename(d.rstrip("/")))
    for (kern, c), v in sorted(agg.items()):
        print(f"   {kern:9s} {c:24s} total {sum(v)/len(v):16.0f}   per tile {sum(v)/len(v)/tiles:10.1f}")
PY
