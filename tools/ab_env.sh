#!/bin/bash
# A/B of environment switches on the default bench line, one bench process per arm, same box:
#   bash tools/ab_env.sh TAG "ENV=1 OTHER=2" "ENV=0" ...   (an empty string = the default arm)
#   BENCH_ARGS="--model large" picks another configuration
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd "$R" || exit 1
i=0
for ARM in "$@"; do
  i=$((i+1))
  env $ARM timeout -k 10 200 python -u bench.py $BENCH_ARGS --steps 20 --warmup 3 --no-cpu-baseline --traffic off --no-roofline \
    > "$O/ab_$i.json" 2> "$O/ab_$i.err" || { echo "arm $i ($ARM) failed"; tail -5 "$O/ab_$i.err"; exit 1; }
  echo "arm $i [$ARM]: $(python3 -c "import json,sys; d=json.load(open('$O/ab_$i.json')); print(d['ms_per_step'], 'ms', d['value'], 'audio-s/s')")"
done
