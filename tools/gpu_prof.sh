#!/bin/bash
# rocprofv3 kernel trace of a short bench run -> per-kernel stats csv under gpurun_out/$1/
set -o pipefail
TAG=${1:-prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 5 --warmup 3 --no-cpu-baseline --traffic off --no-roofline > "$O/prof_bench.json" 2> "$O/prof_bench.err" || { tail -20 "$O/prof_bench.err"; exit 1; }
cat "$O/prof_bench.json"
f=$(find "$O/prof" -name "*kernel_stats.csv" | head -1)
cp "$f" "$O/kernel_stats.csv"
python3 "$R/tools/stats_csv.py" "$O/kernel_stats.csv" 8 45
