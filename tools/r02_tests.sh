set -o pipefail
T=${1:-r02_tests}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 > gpurun_out/$T/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|Error|error" gpurun_out/$T/tests.log | tail -5; grep -A18 "slowest" gpurun_out/$T/tests.log | head -20
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/$T/tests.log | head -80; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err; cat gpurun_out/$T/bench.json
