set -o pipefail
T=${1:-r02_v8}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/$T/tests.log
[ $rc -eq 0 ] || exit 1
for m in 64 3 0; do timeout -k 10 120 python -u tools/ablate.py cfg2 0 $m >> gpurun_out/$T/ablate.txt 2>&1 || exit 1; done
cat gpurun_out/$T/ablate.txt | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py --no-stream --no-cpu > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err; cat gpurun_out/$T/bench.json
