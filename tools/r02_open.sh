set -o pipefail
T=${1:-r02_open}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_open_index.py tests/test_live_index.py tests/test_compaction.py tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread --durations=10 > gpurun_out/$T/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/$T/tests.log | tail -3
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/$T/tests.log | head -100; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err; rc=$?; cat gpurun_out/$T/bench.json; tail -5 gpurun_out/$T/bench.err; exit $rc
