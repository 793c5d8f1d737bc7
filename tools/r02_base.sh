set -o pipefail
mkdir -p gpurun_out/r02_base
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_base/tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/r02_base/tests.log
for m in 64 3 0; do timeout -k 10 120 python -u tools/ablate.py cfg2 0 $m >> gpurun_out/r02_base/ablate.txt 2>&1 || exit 1; done
cat gpurun_out/r02_base/ablate.txt
timeout -k 10 300 python -u bench.py --no-stream > gpurun_out/r02_base/bench.json 2> gpurun_out/r02_base/bench.err; cat gpurun_out/r02_base/bench.json
