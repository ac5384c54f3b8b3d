#!/bin/bash
# Same-box A/B of environment switches on the default bench step (no CPU baseline, no PMC passes), variants
# interleaved over REPS rounds so box drift hits them alike.  Usage (from the repo root, through gpurun):
#   tools/ab_env.sh OUTFILE REPS "ENV=a ENV2=b" "ENV=c" ...
# Each variant's bench line is appended to OUTFILE with its env prefix; a step that fails ends the run.
set -u
OUT=${1:?usage: tools/ab_env.sh OUTFILE REPS VARIANT...}
REPS=${2:?}
shift 2
mkdir -p "$(dirname "$OUT")"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for r in $(seq 1 "$REPS"); do
  for v in "$@"; do
    line=$(env $v timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline --traffic off \
           2> /tmp/ab_err.log)
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant [$v] rc=$rc"; tail -20 /tmp/ab_err.log; exit $rc; fi
    ms=$(python -c "import json,sys; print(json.loads(sys.argv[1])['ms_per_step'])" "$line")
    echo "round $r [$v] ${ms} ms/step" | tee -a "$OUT.txt"
    echo "[$v] $line" >> "$OUT.jsonl"
  done
done
