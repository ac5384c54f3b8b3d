#!/bin/bash
# PMC counters of the attention kernels on the distill-step shape (run on the GPU box)
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/gpurun_out/pmca
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for C in "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_MFMA" "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $C --kernel-include-regex attn -f csv -d $OUT/$i -o run -- python3 $R/tools/attn_bench.py > $OUT/$i.log 2>&1 || { echo "rocprofv3 failed: $C"; tail -5 $OUT/$i.log; exit 1; }
done
cd $R
for f in $(find $OUT -name "*counter_collection.csv" | sort); do
  python3 - "$f" <<'PY'
import csv, sys, collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    d[r["Kernel_Name"].split("(")[0].split("::")[-1]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in d.items():
    print(k, {c: round(sum(x) / len(x)) for c, x in v.items()})
PY
done
