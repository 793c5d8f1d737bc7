#!/bin/bash
# round-3 batch: slice-by-4 tables over 64 LDS banks (16 replicas) vs 32 banks (c232): GPU tests on
# the new layout, k_replay A/B (cfg2, cfg4, cfg3), k_etag_chunk A/B (bench --mode etag)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/r03_b4; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in cfg2 cfg4 cfg3; do
  for v in base c232 base c232; do
    timeout -k 10 120 python -u tools/ablate.py $c 0 $v >> $O/ab.txt 2>&1 || { echo "ab $v failed"; tail -5 $O/ab.txt; exit 1; }
  done
done
grep ablate= $O/ab.txt
for v in "" c232 "" c232; do
  KVREPLAY_VARIANT=$v timeout -k 10 300 python -u bench.py --mode etag > $O/etag_${v:-new}.json 2> $O/etag.err || { echo "etag $v failed"; tail -5 $O/etag.err; exit 1; }
  python -c "import json; d=json.load(open('$O/etag_${v:-new}.json')); print('etag ${v:-new}', d['value'], d['ms_kernel_chunk'], d['roofline']['frac'])" | tee -a $O/ab.txt
done
