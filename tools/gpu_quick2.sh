#!/bin/bash
# Quick GPU pass: selected pytest files, bench (no PMC / CPU baseline), optional probe.
# Usage: bash tools/gpu_quick2.sh TAG "pytest files" [probe]
set -o pipefail
TAG=${1:-q}
TESTS=${2:-tests}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
echo "[q] pytest $TESTS"
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 150 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?
tail -5 "$O/pytest.log"
[ $rc -eq 0 ] || exit $rc
echo "[q] bench"
timeout -k 10 400 python -u bench.py --traffic off --no-cpu-baseline > "$O/bench.json" 2> "$O/bench.err" || { tail -20 "$O/bench.err"; exit 1; }
cat "$O/bench.json"; grep -E "host enqueue|step mode|loss" "$O/bench.err"
if [ -n "$3" ]; then
  echo "[q] probe $3"
  timeout -k 10 200 python -u $3 > "$O/probe.log" 2>&1; echo "probe rc=$?"; tail -8 "$O/probe.log"
fi
