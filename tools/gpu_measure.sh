#!/bin/bash
# One GPU measurement batch, run through gpurun from the repo root:
#   parity tests, the bench line, the rocprofv3 kernel-trace summary of the same bench command,
#   the per-phase cycle breakdown, ablation timings and PMC counters.  Every GPU step has its
#   own time limit and the steps are chained, so the first failure ends the batch.
#   usage: tools/gpu_measure.sh <tag> [tests bench bench3 bench5 prof profc phases ablate vars traffic pmc ...]
set -o pipefail
TAG=${1:-run}; shift
STEPS=${*:-tests bench prof}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R" || exit 1
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 \
        > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -40 "$OUT/tests.log"; exit 1; }
      tail -3 "$OUT/tests.log" ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1 || { echo "smoke failed"; tail -20 "$OUT/smoke.txt"; exit 1; }
      tail -1 "$OUT/smoke.txt" ;;
    bench)
      timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
      cat "$OUT/bench.json" ;;
    bench3)
      timeout -k 10 300 python -u bench.py --config cfg3 --no-cpu --no-open > "$OUT/bench_cfg3.json" 2> "$OUT/bench_cfg3.err" || { echo "bench cfg3 failed"; tail -20 "$OUT/bench_cfg3.err"; exit 1; }
      cat "$OUT/bench_cfg3.json" ;;
    bench5)
      timeout -k 10 400 python -u bench.py --config cfg5 --no-cpu --no-open > "$OUT/bench_cfg5.json" 2> "$OUT/bench_cfg5.err" || { echo "bench cfg5 failed"; tail -20 "$OUT/bench_cfg5.err"; exit 1; }
      cat "$OUT/bench_cfg5.json" ;;
    bench5c)  # cfg5 with its CPU baselines (a 4-segment sample for the faithful port, the shard for the strong one)
      timeout -k 10 900 python -u bench.py --config cfg5 --no-open --no-stream > "$OUT/bench_cfg5_cpu.json" 2> "$OUT/bench_cfg5_cpu.err" || { echo "bench cfg5 cpu failed"; tail -20 "$OUT/bench_cfg5_cpu.err"; exit 1; }
      cat "$OUT/bench_cfg5_cpu.json" ;;
    etag)
      timeout -k 10 300 python -u bench.py --mode etag > "$OUT/bench_etag.json" 2> "$OUT/bench_etag.err" || { echo "bench etag failed"; tail -20 "$OUT/bench_etag.err"; exit 1; }
      cat "$OUT/bench_etag.json" ;;
    profe)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profe" -o run -- \
        python "$R/bench.py" --mode etag > "$OUT/profe.log" 2>&1) || { echo "rocprof etag failed"; tail -20 "$OUT/profe.log"; exit 1; }
      find "$OUT/profe" -name '*kernel_stats.csv' -exec cat {} \; ;;
    prof)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
        python "$R/bench.py" --no-cpu --no-stream --no-open > "$OUT/prof.log" 2>&1) || { echo "rocprof failed"; tail -20 "$OUT/prof.log"; exit 1; }
      find "$OUT/prof" -name '*kernel_stats.csv' -exec cat {} \; ;;
    trace)    # kernel + memory-copy timeline of the headline step (tools/trace_gaps.py): the gaps around k_replay
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$OUT/trace" -o run -- \
        python "$R/bench.py" --no-cpu --no-stream --no-open --steps 20 > "$OUT/trace.log" 2>&1) || { echo "trace failed"; tail -20 "$OUT/trace.log"; exit 1; }
      python "$R/tools/trace_gaps.py" "$OUT/trace" > "$OUT/trace_gaps.txt" 2>&1; cat "$OUT/trace_gaps.txt" ;;
    profc)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profc" -o run -- \
        python "$R/bench.py" --mode compact --steps 5 --warmup 2 > "$OUT/profc.log" 2>&1) || { echo "rocprof compact failed"; tail -20 "$OUT/profc.log"; exit 1; }
      find "$OUT/profc" -name '*kernel_stats.csv' -exec cat {} \; ;;
    profi)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profi" -o run -- \
        python "$R/tools/prof_index.py" cfg2 5 > "$OUT/profi.log" 2>&1) || { echo "rocprof index failed"; tail -20 "$OUT/profi.log"; exit 1; }
      cat "$OUT/profi.log"; find "$OUT/profi" -name '*kernel_stats.csv' -exec cat {} \; ;;
    profi2)   # the same with the claim kernel preloading key prefixes (timing knob)
      (cd /tmp && KVR_CLAIM_PRELOAD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profi2" -o run -- \
        python "$R/tools/prof_index.py" cfg2 5 > "$OUT/profi2.log" 2>&1) || { echo "rocprof index2 failed"; tail -20 "$OUT/profi2.log"; exit 1; }
      cat "$OUT/profi2.log"; find "$OUT/profi2" -name '*kernel_stats.csv' -exec grep -E "fold|k_live|index" {} \; ;;
    benchc)
      timeout -k 10 300 python -u bench.py --mode compact > "$OUT/bench_compact.json" 2> "$OUT/bench_compact.err" || { echo "bench compact failed"; tail -20 "$OUT/bench_compact.err"; exit 1; }
      cat "$OUT/bench_compact.json" ;;
    phases)
      timeout -k 10 240 python -u tools/prof_phases.py cfg2 > "$OUT/phases_cfg2.txt" 2>&1 || { echo "phases failed"; tail -20 "$OUT/phases_cfg2.txt"; exit 1; }
      cat "$OUT/phases_cfg2.txt" ;;
    phases4)  # the cfg4 shape (50 % DEL: two record lengths, the framing's hard case)
      timeout -k 10 240 python -u tools/prof_phases.py cfg4 > "$OUT/phases_cfg4.txt" 2>&1 || { echo "phases4 failed"; tail -20 "$OUT/phases_cfg4.txt"; exit 1; }
      cat "$OUT/phases_cfg4.txt" ;;
    bench4)
      timeout -k 10 300 python -u bench.py --config cfg4 --no-cpu --no-open --no-stream > "$OUT/bench_cfg4.json" 2> "$OUT/bench_cfg4.err" || { echo "bench cfg4 failed"; tail -20 "$OUT/bench_cfg4.err"; exit 1; }
      cat "$OUT/bench_cfg4.json" ;;
    ablate)
      for m in ${MASKS:-0 1 2 3 7}; do
        timeout -k 10 120 python -u tools/ablate.py cfg2 0 $m >> "$OUT/ablate_cfg2.txt" 2>&1 || { echo "ablate failed"; tail -20 "$OUT/ablate_cfg2.txt"; exit 1; }
      done
      cat "$OUT/ablate_cfg2.txt" ;;
    vars)     # build.py VARIANTS named in $VARS, timed one process each (cfg in $VCFG)
      for v in ${VARS:-base}; do
        timeout -k 10 120 python -u tools/ablate.py ${VCFG:-cfg2} 0 $v >> "$OUT/vars_${VCFG:-cfg2}.txt" 2>&1 || { echo "variant $v failed"; tail -20 "$OUT/vars_${VCFG:-cfg2}.txt"; exit 1; }
      done
      cat "$OUT/vars_${VCFG:-cfg2}.txt" ;;
    foldv)    # tools/prof_index.py under each build pair named in $FOLDV (build.py build_variant_pair)
      for v in ${FOLDV:-base}; do
        echo "variant $v" >> "$OUT/foldv.txt"
        KVREPLAY_VARIANT=$v timeout -k 10 120 python -u tools/prof_index.py ${VCFG:-cfg2} 6 >> "$OUT/foldv.txt" 2>&1 || { echo "foldv $v failed"; tail -20 "$OUT/foldv.txt"; exit 1; }
      done
      cat "$OUT/foldv.txt" ;;
    traffic)
      timeout -k 10 600 python -u tools/pmc_traffic.py > "$OUT/traffic.log" 2>&1 || { echo "traffic failed"; tail -20 "$OUT/traffic.log"; exit 1; }
      cp gpurun_out/pmc_traffic.json "$OUT/pmc_traffic.json" && tail -1 "$OUT/traffic.log" ;;
    pmc)
      timeout -k 10 900 bash tools/pmc.sh "$OUT/pmc" --no-cpu --no-stream --steps 2 --warmup 1 > "$OUT/pmc.txt" 2>&1 || { echo "pmc failed"; tail -20 "$OUT/pmc.txt"; exit 1; }
      cat "$OUT/pmc.txt" ;;
    pmce)     # PMC counters of the batch ETag bench (k_etag_chunk)
      timeout -k 10 900 bash tools/pmc.sh "$OUT/pmce" --mode etag --steps 2 --warmup 1 > "$OUT/pmce.txt" 2>&1 || { echo "pmce failed"; tail -20 "$OUT/pmce.txt"; exit 1; }
      cat "$OUT/pmce.txt" ;;
    pmc4)     # PMC counters of the cfg4-shape bench (two record lengths, the hop loop's case)
      timeout -k 10 900 bash tools/pmc.sh "$OUT/pmc4" --config cfg4 --no-cpu --no-stream --no-open --steps 2 --warmup 1 > "$OUT/pmc4.txt" 2>&1 || { echo "pmc4 failed"; tail -20 "$OUT/pmc4.txt"; exit 1; }
      cat "$OUT/pmc4.txt" ;;
    ldpat)    # tools/ldpat.hip: the load-structure ceiling of the tile loop (built here beforehand)
      timeout -k 10 180 ./tools/ldpat > "$OUT/ldpat.txt" 2>&1 || { echo "ldpat failed"; tail -20 "$OUT/ldpat.txt"; exit 1; }
      cat "$OUT/ldpat.txt" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "batch $TAG done"
