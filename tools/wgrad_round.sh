# wgrad (mn x mn, split-K) shapes: register-staged kernel vs ring paths, then GEMM tests
set -o pipefail
mkdir -p gpurun_out/wg
O=gpurun_out/wg/out.txt; [ -n "$KEEP" ] || rm -f $O
for sh in 768,3072,7984,0,0,3 3072,768,7984,0,0,3 2304,768,7984,0,0,4 768,768,7984,0,0,14 512,1536,255984,0,0,10 7984,3072,768,1,0,1; do
  for p in ${PATHS:-small mid mid8mn}; do
    echo -n "$p nt=${DPH_GEMM_SMALL_NT:-256} " >> $O
    DPH_LIB_PATH=ab/abl0.so DPH_GEMM_PATH=$p timeout -k 10 60 python tools/ablate_gemm.py time ${sh//,/ } 2>&1 | grep -v amdgpu.ids >> $O || exit 1
  done
done
cat $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/wg/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/wg/pytest.log; exit $rc
