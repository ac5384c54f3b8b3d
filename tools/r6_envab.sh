#!/bin/bash
# same-box bench A/B of one environment switch: tools/r6_envab.sh OUTDIR "ENV=VAL ..." [rounds]
# (default vs the given env, interleaved; 30 timed steps each, no CPU baseline / PMC passes)
set -u
OUT=${1:?outdir}; ENVB=${2:?env}; R=${3:-2}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for i in $(seq 1 $R); do
  for v in A B; do
    if [ $v = A ]; then E=""; else E="$ENVB"; fi
    env $E timeout -k 10 300 python -u bench.py --steps 30 --no-cpu-baseline --traffic off > "$OUT/$v$i.json" 2> "$OUT/$v$i.log"
    rc=$?
    echo "$v$i [$E] rc=$rc $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$v$i.json" | head -1)"
    if [ $rc -ne 0 ]; then tail -20 "$OUT/$v$i.log"; exit $rc; fi
  done
done
