set -o pipefail
mkdir -p gpurun_out/wl1
timeout -k 10 300 python -u -m pytest tests/test_wavlm_gpu.py "tests/test_parity_gpu.py::test_distill_step_vs_reference" -x -v -s --timeout 120 --timeout-method thread > gpurun_out/wl1/wavlm.log 2>&1 || { tail -60 gpurun_out/wl1/wavlm.log; exit 1; }
grep -E "PASS|FAIL|rel-L2" gpurun_out/wl1/wavlm.log | tail -30
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/wl1/all.log 2>&1 || { tail -40 gpurun_out/wl1/all.log; exit 1; }
tail -3 gpurun_out/wl1/all.log
