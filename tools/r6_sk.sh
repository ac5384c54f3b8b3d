#!/bin/bash
# stream-K GEMM: parity tests, then the tile / stream-K A/B on the step's projection shapes
set -u
OUT=${1:?outdir}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_sk_gpu.py -x -v --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 "$OUT/tests.log"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/pp_tile_ab.py 5 auto sk0 skall 16 15 > "$OUT/ab.txt" 2>&1
rc=$?; echo "ab rc=$rc"; cat "$OUT/ab.txt"; exit $rc
