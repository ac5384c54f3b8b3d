set -o pipefail
mkdir -p gpurun_out/c0b
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/c0b/pytest.log 2>&1; rc=$?; tail -15 gpurun_out/c0b/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 2 3; do DPH_C0B_VARIANT=$v timeout -k 10 120 python -u tools/c0b_bench.py || exit 1; done
