#!/bin/bash
# WavLM: GPU tests, WavLM-Base bench (graph replay), kernel-trace profile of the same bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${TAG:-wl2}
mkdir -p "$O"
cd "$R" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_wavlm_gpu.py -x -v -s --timeout 120 --timeout-method thread > "$O/wavlm.log" 2>&1 || { tail -40 "$O/wavlm.log"; exit 1; }
grep -E "PASS|FAIL" "$O/wavlm.log" | tail
timeout -k 10 400 python -u bench.py --model wavlm-base --no-cpu-baseline --traffic off > "$O/bench_wavlm.json" 2> "$O/bench_wavlm.err" || { tail -30 "$O/bench_wavlm.err"; exit 1; }
cat "$O/bench_wavlm.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o run -- python3 "$R/bench.py" --model wavlm-base --steps 5 --warmup 3 --no-cpu-baseline --traffic off > "$O/prof_bench.json" 2> "$O/prof_bench.err" || { tail -30 "$O/prof_bench.err"; exit 1; }
cat "$O/prof_bench.json"
