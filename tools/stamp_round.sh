set -o pipefail
mkdir -p gpurun_out/st
for lib in ${LIBS:-stamp}; do
for sh in ${SHAPES:-"7984,3072,768 7984,768,3072"}; do
echo "== $lib $sh" >> gpurun_out/st/out.txt
DPH_LIB_PATH=ab/$lib.so DPH_GEMM_PATH=mid timeout -k 10 60 python tools/stamp_gemm.py time ${sh//,/ } 2>&1 | grep -v "amdgpu.ids\|decile" >> gpurun_out/st/out.txt || exit 1
done; done
