#!/bin/bash
# round-3 batch: open-index + compaction GPU tests, then k_replay ablations on the cfg4 shape
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out/r03_b1
timeout -k 10 400 python -u -m pytest tests/test_open_index.py tests/test_compaction.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/r03_b1/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03_b1/tests.log; exit 1; }
tail -2 gpurun_out/r03_b1/tests.log
for m in 0 1 2 4 8 16 32 64; do
  timeout -k 10 120 python -u tools/ablate.py cfg4 0 $m >> gpurun_out/r03_b1/ablate_cfg4.txt 2>&1 || { echo "ablate $m failed"; tail -5 gpurun_out/r03_b1/ablate_cfg4.txt; exit 1; }
done
grep ablate= gpurun_out/r03_b1/ablate_cfg4.txt
