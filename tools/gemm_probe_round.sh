set -o pipefail
mkdir -p gpurun_out/g2
for sh in "7984 3072 768" "7984 768 3072" "7984 768 768" "7984 2304 768"; do
 for n in 0 5 6; do for p in mid big; do
  DPH_LIB_PATH=ab/abl$n.so DPH_GEMM_PATH=$p timeout -k 10 60 python tools/ablate_gemm.py time $sh 2>/dev/null | sed "s/$/ path=$p/" >> gpurun_out/g2/ablate.txt || exit 1
 done; done
done
