#!/bin/bash
# split-graph teacher concurrency: graph tests, then bench A/B (split vs one graph with the fork inside)
set -u
OUT=${1:?outdir}; mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
timeout -k 10 600 python -u -m pytest tests/test_graph_gpu.py tests/test_fullshape_gpu.py -x -v --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 "$OUT/tests.log"; if [ $rc -ne 0 ]; then grep -E "Error|assert" "$OUT/tests.log" | head -20; exit $rc; fi
run_bench() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 30 --no-cpu-baseline --traffic off > "$OUT/$name.json" 2> "$OUT/$name.log"
  local rc=$?; echo "$name rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$name.json") $(grep -o '"host": {[^}]*}' "$OUT/$name.json")"
  if fatal $rc; then tail -20 "$OUT/$name.log"; exit $rc; fi
}
run_bench split
run_bench onegraph DPH_GRAPH_SPLIT=0
run_bench split2
run_bench onegraph2 DPH_GRAPH_SPLIT=0
