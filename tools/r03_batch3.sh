#!/bin/bash
# round-3 batch: k_etag_chunk with the 64-KiB LDS layout (2 workgroups of 10 waves per CU) against
# the same layout at one 16-wave workgroup (ew16) and round 2's layout (eold); etag tests first
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/r03_b3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_etag.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in "" ew16 eold "" ew16 eold; do
  KVREPLAY_VARIANT=$v timeout -k 10 300 python -u bench.py --mode etag > $O/etag_${v:-new}.json 2> $O/etag.err || { echo "etag $v failed"; tail -5 $O/etag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/etag_${v:-new}.json')); print('etag ${v:-new}', d['value'], d['ms_kernel_chunk'], d['roofline']['frac'])" | tee -a $O/ab.txt
done
