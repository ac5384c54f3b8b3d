#!/bin/bash
# A/B timing on the GPU box: the in-tree library vs another build of it (DPH_LIB_PATH), on the GEMM shapes of
# the step (tools/gemm_bench.py) and on the whole bench step.  usage: bash tools/ab_round.sh TAG OTHER_LIB [gemm|attn|step ...]
set -o pipefail
TAG=$1; OTHER=$2; shift 2
WHAT=${*:-gemm step}
O=gpurun_out/$TAG; mkdir -p $O
for W in $WHAT; do
  for L in new old; do
    if [ $L = old ]; then export DPH_LIB_PATH=$OTHER; else unset DPH_LIB_PATH; fi
    case $W in
      gemm) timeout -k 10 300 python -u tools/gemm_bench.py > $O/gemm_$L.txt 2>&1 || { tail -20 $O/gemm_$L.txt; exit 1; } ;;
      attn) timeout -k 10 300 python -u tools/attn_bench.py > $O/attn_$L.txt 2>&1 || { tail -20 $O/attn_$L.txt; exit 1; } ;;
      step) timeout -k 10 300 python -u bench.py --steps 20 --no-cpu-baseline --traffic off > $O/step_$L.json 2> $O/step_$L.err || { tail -20 $O/step_$L.err; exit 1; } ;;
    esac
  done
done
for W in $WHAT; do
  case $W in
    gemm|attn) paste -d'\n' $O/${W}_new.txt $O/${W}_old.txt | sed 's/^/  /' ;;
    step) for L in new old; do python3 -c "import json,sys; d=json.load(open('$O/step_$L.json')); print('$L', d['ms_per_step'], 'ms', d['roofline']['avg_launch_us'], 'us/launch frac', d['roofline']['frac'])"; done ;;
  esac
done
