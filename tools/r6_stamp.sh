set -u
OUT=gpurun_out/r6_stamp1; mkdir -p $OUT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
DPH_LIB_PATH=ab/stamp_sk.so timeout -k 10 120 python -u tools/stamp_sk.py time 7984 3072 768 gelu > $OUT/ffn1.txt 2>&1 || { cat $OUT/ffn1.txt; exit 1; }
DPH_LIB_PATH=ab/stamp_sk.so timeout -k 10 120 python -u tools/stamp_sk.py time 7984 2304 768 > $OUT/qkv.txt 2>&1 || { cat $OUT/qkv.txt; exit 1; }
DPH_LIB_PATH=ab/stamp_sk.so timeout -k 10 120 python -u tools/stamp_sk.py time 8192 8192 8192 > $OUT/big.txt 2>&1 || { cat $OUT/big.txt; exit 1; }
cat $OUT/*.txt
timeout -k 10 300 python -u tools/pp_tile_ab.py 3 auto sk0 12 16 15 > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; exit $rc
