#!/bin/bash
# FETCH_SIZE (raw KiB, mean per k_replay main-pass dispatch) of A/B builds over tools/ablate.py
# $PCFG (default cfg2): one rocprofv3 --pmc pass per build.
#   usage: tools/fetch_variants.sh <outdir> <build names...>
set -o pipefail
OUT=$(mkdir -p "$1" && cd "$1" && pwd); shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
for m in "$@"; do
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/$m" -o pmc -- python "$R/tools/ablate.py" ${PCFG:-cfg2} 0 $m \
    > "$OUT/$m.log" 2>&1 || { echo "build $m failed"; tail -5 "$OUT/$m.log"; exit 1; }
done
python - "$OUT" "$@" <<'PY'
import csv, glob, sys
out = sys.argv[1]
for m in sys.argv[2:]:
    rows = []
    for f in glob.glob(f"{out}/{m}/**/*counter_collection.csv", recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if "k_replay" in r["Kernel_Name"]]
    big = max(int(r["Grid_Size"]) for r in rows)
    v = [float(r["Counter_Value"]) for r in rows if int(r["Grid_Size"]) == big]
    print(f"{m}: FETCH_SIZE raw KiB per dispatch {sum(v) / len(v):.0f} (n={len(v)})")
PY
