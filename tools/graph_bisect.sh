#!/bin/bash
# runs the bisect modes in order, stopping at the first failure
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/bis; mkdir -p "$O"; cd "$R" || exit 1
for m in gemm memset teacher student fwdbwd full; do
  timeout -k 10 150 python -u tools/graph_bisect.py $m > "$O/$m.log" 2>&1
  rc=$?
  echo "mode $m rc=$rc"; grep "^\[" "$O/$m.log" | tail -3
  [ $rc -eq 0 ] || { grep -v "^  File" "$O/$m.log" | tail -15; exit $rc; }
done
