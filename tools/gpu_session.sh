#!/bin/bash
# One GPU-box session (run through gpurun from the repo root): the -m gpu suite, then the default bench line with
# its PMC traffic passes and CPU baseline, then a rocprofv3 kernel-trace summary of a short bench run.  Every GPU
# step runs under its own time limit; a fault, abort or time-out (exit status >= 124, or a signal) ends the session
# there.  Usage: tools/gpu_session.sh OUTDIR [tests|bench|prof ...]   (default: tests bench prof)
set -u
OUT=${1:?usage: tools/gpu_session.sh OUTDIR [steps]}
shift
STEPS=${*:-tests bench prof}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0

fatal() {  # exit statuses that mean the GPU step crashed or hung
  local rc=$1
  [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]
}

for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=30 --timeout 300 --timeout-method thread \
        > "$OUT/tests.log" 2>&1
      rc=$?; echo "tests rc=$rc"; tail -3 "$OUT/tests.log"
      if fatal $rc; then exit $rc; fi ;;
    bench)
      DPH_BENCH_PMC_DIR="$OUT/pmc" timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.log"
      rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"
      if [ $rc -ne 0 ]; then tail -20 "$OUT/bench.log"; exit $rc; fi ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- \
        python -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --traffic off > "$OUT/prof_bench.json" 2> "$OUT/prof.log"
      rc=$?; echo "prof rc=$rc"
      if [ $rc -ne 0 ]; then tail -20 "$OUT/prof.log"; exit $rc; fi
      find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \; ;;
    *)
      echo "unknown step $s"; exit 2 ;;
  esac
done
