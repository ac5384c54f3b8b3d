set -o pipefail
O=gpurun_out/r3_s4; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -3 $O/t.log; [ $rc -eq 0 ] || { grep -E "^(FAILED|E )" $O/t.log | head; exit $rc; }
timeout -k 10 300 python -u tools/gemm_ab.py auto pp256 pp128x192 pp128 pp128x256 > $O/gemm_ab.log 2>&1; rc=$?; cut -c1-300 $O/gemm_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline --traffic off > $O/bench.json 2> $O/bench.err; rc=$?; tail -3 $O/bench.err; exit $rc
