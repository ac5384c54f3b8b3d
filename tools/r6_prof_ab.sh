#!/bin/bash
# same-box kernel-stats A/B of one environment switch: tools/r6_prof_ab.sh OUTDIR "ENV=VAL"
# (rocprofv3 kernel trace of bench.py --steps 8 --warmup 3, default then with the env)
set -u
OUT=${1:?outdir}; ENVB=${2:?env}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for v in A B; do
  if [ $v = A ]; then E=""; else E="$ENVB"; fi
  for kv in $E; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/$v" -o run -- \
    python -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --traffic off > "$OUT/$v.json" 2> "$OUT/$v.log"
  rc=$?
  echo "$v [$E] rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$v.log"; exit $rc; fi
done
