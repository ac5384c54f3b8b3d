#!/bin/bash
# quick GPU check: selected tests + GEMM microbench.  usage: bash tools/gpu_quick.sh TAG "pytest selection"
set -o pipefail
TAG=$1; SEL=${2:-tests}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u tools/gemm_bench.py > $O/gemm_bench.txt 2>&1 || { tail -20 $O/gemm_bench.txt; exit 1; }
cat $O/gemm_bench.txt | grep -v amdgpu.ids
if [ -n "$BENCH" ]; then timeout -k 10 300 python -u bench.py --no-cpu-baseline --traffic off > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }; cat $O/bench.json; grep "host enqueue" $O/bench.err; fi
