#!/bin/bash
# per-block timelines of the ping-pong tile kernels on the step's K = 768 projection shapes (tools/stamp_pp.py)
set -u
OUT=gpurun_out/r6_stamp_pp; mkdir -p $OUT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in "16 7984 3072 768" "15 7984 3072 768" "15 7984 2304 768" "16 7984 2304 768" "15 7984 768 768 resid" "15 7984 768 3072 resid"; do
  set -- $cfg
  DPH_LIB_PATH=ab/stamp_pp.so DPH_PP_FORCE=$1 timeout -k 10 120 python -u tools/stamp_pp.py time $2 $3 $4 ${5:-} >> $OUT/stamps.txt 2>&1 || { tail -5 $OUT/stamps.txt; exit 1; }
done
grep -v amdgpu.ids $OUT/stamps.txt
