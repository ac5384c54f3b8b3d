#!/bin/bash
# Round-6 GPU A/B session: each step under its own time limit; a crash / time-out ends the session.
# Usage: tools/r6_ab.sh OUTDIR
set -u
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
run_bench() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 30 --no-cpu-baseline --traffic off > "$OUT/$name.json" 2> "$OUT/$name.log"
  local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep 'host loop' "$OUT/$name.log")"
  if fatal $rc; then tail -20 "$OUT/$name.log"; exit $rc; fi
}
timeout -k 10 400 python -u -m pytest tests/test_graph_gpu.py -k "deferred" -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 "$OUT/tests.log"; if fatal $rc; then exit $rc; fi
run_bench default
run_bench teacher_serial DPH_TEACHER_STREAM=0
run_bench default2
run_bench teacher_serial2 DPH_TEACHER_STREAM=0
