# quick A/B of ring GEMM tiles on step shapes (production library), then GEMM tests
set -o pipefail
mkdir -p gpurun_out/abl2
O=gpurun_out/abl2/out.txt
rm -f $O
for sh in ${SHAPES:-7984,768,3072 7984,768,768 7984,3072,768 7984,2304,768}; do
  for p in ${PATHS:-mid half}; do
  for L in ${LIBS:-abl0}; do
    echo -n "$p " >> $O
    DPH_LIB_PATH=ab/$L.so DPH_GEMM_PATH=$p timeout -k 10 60 python tools/ablate_gemm.py time ${sh//,/ } 2>&1 | grep -v amdgpu.ids >> $O || exit 1
  done
  done
done
cat $O
[ -n "$NOTEST" ] && exit 0
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/abl2/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/abl2/pytest.log; exit $rc
