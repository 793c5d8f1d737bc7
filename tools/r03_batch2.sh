#!/bin/bash
# round-3 batch: GPU parity tests, then A/B: the scalar path's key preload (cfg4, cfg2) and
# k_etag_chunk's step-input carry (bench --mode etag under the xc0 build pair)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
O=gpurun_out/r03_b2; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in base kpre0 base kpre0; do
  timeout -k 10 120 python -u tools/ablate.py cfg4 0 $v >> $O/ab.txt 2>&1 || { echo "ab $v failed"; tail -5 $O/ab.txt; exit 1; }
done
for v in base kpre0; do
  timeout -k 10 120 python -u tools/ablate.py cfg2 0 $v >> $O/ab.txt 2>&1 || { echo "ab $v failed"; tail -5 $O/ab.txt; exit 1; }
done
grep ablate= $O/ab.txt
for v in "" xc0 "" xc0; do
  KVREPLAY_VARIANT=$v timeout -k 10 300 python -u bench.py --mode etag > $O/etag_${v:-base}.json 2> $O/etag.err || { echo "etag $v failed"; tail -5 $O/etag.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/etag_${v:-base}.json')); print('etag ${v:-base}', d['value'], d['ms_kernel_chunk'], d['roofline']['frac'])"
done
