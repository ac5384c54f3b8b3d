set -o pipefail
mkdir -p gpurun_out/abl
O=gpurun_out/abl/out.txt
for sh in "255984 512 1536 big" "7984 3072 768 mid" "7984 768 3072 mid"; do
  set -- $sh
  for v in 0 5 1 2 4 6; do
    DPH_LIB_PATH=ab/abl$v.so DPH_GEMM_PATH=$4 timeout -k 10 60 python tools/ablate_gemm.py time $1 $2 $3 2>&1 | grep -v amdgpu.ids >> $O || exit 1
  done
  DPH_LIB_PATH=ab/stamp.so DPH_GEMM_PATH=$4 timeout -k 10 60 python tools/stamp_gemm.py time $1 $2 $3 2>&1 | grep -v "amdgpu.ids\|decile" >> $O || exit 1
done
cat $O
