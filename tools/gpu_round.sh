#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench (with PMC traffic + CPU baseline), kernel-trace profile.
# Usage (from the repo root on the GPU box): bash tools/gpu_round.sh [tag]
set -o pipefail
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
echo "[gpu_round] pytest -m gpu"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || { tail -30 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
echo "[gpu_round] smoke"
timeout -k 10 120 python -u __graft_entry__.py smoke > "$O/smoke.log" 2>&1 || { tail -30 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
echo "[gpu_round] bench"
timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -30 "$O/bench.err"; exit 1; }
cat "$O/bench.json"
echo "[gpu_round] rocprofv3 kernel trace"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 5 --warmup 3 --no-cpu-baseline --traffic off > "$O/prof_bench.json" 2> "$O/prof_bench.err" || { tail -30 "$O/prof_bench.err"; exit 1; }
cat "$O/prof_bench.json"
echo "[gpu_round] done"
