#!/bin/bash
# PMC counters of the GEMM paths on one shape (run on the GPU box).
# usage: bash tools/pmc_gemm.sh M N K [paths] [counter-set ...]
#   paths: "big small" (default); each counter set is one rocprofv3 pass
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/pmcg
rm -rf $OUT; mkdir -p $OUT
M=$1; N=$2; K=$3; shift 3
PATHS=${1:-"big small"}; [ $# -gt 0 ] && shift
SETS=("$@")
[ ${#SETS[@]} -eq 0 ] && SETS=("SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA" "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" "GRBM_GUI_ACTIVE")
cd /tmp && export TMPDIR=/tmp
i=0
for P in $PATHS; do
  for C in "${SETS[@]}"; do
    i=$((i+1))
    DPH_GEMM_PATH=$P timeout -k 10 120 rocprofv3 --pmc $C -f csv -d $OUT/$P-$i -o run -- python3 $R/tools/gemm_one.py $M $N $K 3 > $OUT/$P-$i.log 2>&1 || { echo "rocprofv3 failed: $P $C"; tail -5 $OUT/$P-$i.log; exit 1; }
  done
done
cd $R
for f in $(find $OUT -name "*counter_collection.csv" | sort); do
  python3 - "$f" <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "gemm" in r["Kernel_Name"]:
        d[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[1].split("/")[-2], {k: round(sum(v) / len(v)) for k, v in d.items()})
PY
done
