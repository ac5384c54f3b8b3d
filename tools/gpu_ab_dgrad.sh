set -o pipefail
bash tools/gpu_quick2.sh g3 "tests" || exit 1
echo "[ab] DPH_DGRAD_T=0"
DPH_DGRAD_T=0 timeout -k 10 400 python -u bench.py --traffic off --no-cpu-baseline > gpurun_out/g3/bench_t0.json 2> gpurun_out/g3/bench_t0.err || exit 1
grep -E "loss" gpurun_out/g3/bench_t0.err
