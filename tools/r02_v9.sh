set -o pipefail
T=$1; shift
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/$T/tests.log
[ $rc -eq 0 ] || exit 1
for v in "$@"; do timeout -k 10 120 python -u tools/ablate.py cfg2 0 $v >> gpurun_out/$T/var.txt 2>&1 || { tail -5 gpurun_out/$T/var.txt; exit 1; }; done
grep -v amdgpu.ids gpurun_out/$T/var.txt
timeout -k 10 300 python -u bench.py --no-stream --no-cpu > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err; cat gpurun_out/$T/bench.json
