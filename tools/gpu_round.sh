#!/bin/bash
# One GPU-box pass (run from the repo root on the box via gpurun):
#   bash tools/gpu_round.sh TAG [phase ...]
# phases (default: parity tests smoke bench prof):
#   parity  -- tests/test_parity_gpu.py with -s (per-fixture error tables), all cases run; a failure ends the script
#   tests   -- the whole -m gpu suite, -x
#   testsall -- the whole -m gpu suite without -x (every failure listed; a failing test does not end the script)
#   smoke   -- __graft_entry__.smoke()
#   bench   -- bench.py default line (PMC traffic passes + CPU baseline)
#   prof    -- rocprofv3 --kernel-trace --stats of a short bench run -> kernel_stats.csv
#   gemmtests -- tests/test_gemm_gpu.py (every GEMM path)
#   wgrad   -- tools/wgrad_ab.py (weight-gradient GEMMs: ppw plan vs the register-staged kernel)
#   pmcattn -- rocprofv3 --pmc passes over the attention kernels (tools/attn_bench.py)
#   pmcgemm -- the same over the dominant GEMM shape (7984 x 3072 x 768, tools/gemm_one.py)
#   pmcgemmx -- PMC of the 128 x 192 tile (FFN2 shape, 8192^3) and the 256 x 256 tile (8192^3)
#   pmcconv0 -- the same over the conv0 GroupNorm kernels (tools/conv0_bench.py)
# Every GPU step runs under its own timeout; the first failing step ends the script.
set -o pipefail
TAG=${1:-run}; shift
PHASES=${*:-parity tests smoke bench prof}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
PYT="python -u -m pytest --timeout 120 --timeout-method thread"
# pmc_run TAG KERNEL_REGEX CMD...: two rocprofv3 --pmc passes (8 SQ + 2 GRBM counters each fit one pass) and a
# kernel-trace pass of the same command, summarised by tools/pmc_summary.py into $O/TAG_summary.txt
pmc_run() {
  local tag=$1 rx=$2; shift 2
  local i=0
  for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$rx" -f csv \
      -d "$O/$tag/$i" -o run -- "$@" > "$O/${tag}_$i.log" 2>&1) || { echo "rocprofv3 pass $i failed"; tail -5 "$O/${tag}_$i.log"; return 1; }
  done
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats --kernel-include-regex "$rx" \
    -f csv -d "$O/$tag/trace" -o run -- "$@" > "$O/${tag}_trace.log" 2>&1) || { echo "trace pass failed"; return 1; }
  python3 tools/pmc_summary.py "$O/$tag" > "$O/${tag}_summary.txt" && cat "$O/${tag}_summary.txt"
  f=$(find "$O/$tag/trace" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" "$O/${tag}_kernel_stats.csv"
  return 0
}
for P in $PHASES; do
  echo "[gpu_round] $P $(date +%T)"
  case $P in
    parity)
      timeout -k 10 300 $PYT tests/test_parity_gpu.py -m gpu -v -s > "$O/parity.log" 2>&1
      rc=$?; grep -E "passed|failed|Error" "$O/parity.log" | tail -5
      [ $rc -eq 0 ] || exit $rc ;;
    tests)
      timeout -k 10 900 $PYT tests -m gpu -x -q > "$O/pytest_gpu.log" 2>&1 || { tail -40 "$O/pytest_gpu.log"; exit 1; }
      tail -3 "$O/pytest_gpu.log" ;;
    testsall)
      timeout -k 10 900 $PYT tests -m gpu -q > "$O/pytest_gpu.log" 2>&1; rc=$?
      grep -E "^(FAILED|ERROR)" "$O/pytest_gpu.log" | head -20; tail -2 "$O/pytest_gpu.log"
      [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc ;;
    smoke)
      timeout -k 10 180 python -u __graft_entry__.py smoke > "$O/smoke.log" 2>&1 || { tail -30 "$O/smoke.log"; exit 1; }
      tail -1 "$O/smoke.log" ;;
    bench)
      timeout -k 10 700 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail -30 "$O/bench.err"; exit 1; }
      cat "$O/bench.json" ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o run \
        -- python3 "$R/bench.py" --steps 5 --warmup 3 --no-cpu-baseline --traffic off \
        > "$O/prof_bench.json" 2> "$O/prof_bench.err") || { tail -30 "$O/prof_bench.err"; exit 1; }
      cat "$O/prof_bench.json"
      f=$(find "$O/prof" -name "*kernel_stats.csv" | head -1)
      cp "$f" "$O/kernel_stats.csv" && python3 tools/stats_csv.py "$O/kernel_stats.csv" 8 40 ;;
    gemmtests)
      timeout -k 10 600 $PYT tests/test_gemm_gpu.py -m gpu -x -q > "$O/gemm_tests.log" 2>&1 || { tail -40 "$O/gemm_tests.log"; exit 1; }
      tail -2 "$O/gemm_tests.log" ;;
    wgrad)
      timeout -k 10 300 python -u tools/wgrad_ab.py > "$O/wgrad_ab.log" 2>&1 || { tail -30 "$O/wgrad_ab.log"; exit 1; }
      cut -c1-220 "$O/wgrad_ab.log" ;;
    pmcattn)
      pmc_run pmcattn attn python3 "$R/tools/attn_bench.py" || exit 1 ;;
    pmcgemm)
      pmc_run pmcgemm gemm python3 "$R/tools/gemm_one.py" 7984 3072 768 5 || exit 1 ;;
    pmcgemmx)
      # the 128 x 192 tile on the FFN2 projection shape and on 8192^3, the 256 x 256 tile on 8192^3
      for cfg in "15 7984 768 3072" "15 8192 8192 8192" "12 8192 8192 8192"; do
        set -- $cfg
        (export DPH_PP_FORCE=$1; pmc_run "pmcgemm_$1_$2x$3x$4" gemm python3 "$R/tools/gemm_one.py" $2 $3 $4 5) || exit 1
      done ;;
    pmcconv0)
      pmc_run pmcconv0 conv0 python3 "$R/tools/conv0_bench.py" 0 3 || exit 1 ;;
    *) echo "unknown phase $P"; exit 2 ;;
  esac
done
echo "[gpu_round] done $(date +%T)"
