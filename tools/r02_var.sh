set -o pipefail
T=$1; shift
mkdir -p gpurun_out/$T
for v in "$@"; do timeout -k 10 120 python -u tools/ablate.py cfg2 0 $v >> gpurun_out/$T/var.txt 2>&1 || { tail -5 gpurun_out/$T/var.txt; exit 1; }; done
grep -v amdgpu.ids gpurun_out/$T/var.txt
