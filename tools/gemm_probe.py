import sys
import torch
sys.path.insert(0, ".")
from tools.gemm_bench import run
M = 16 * 499
for Kd in (64, 128, 256, 768, 1536, 3072):
    run(f"N768 K{Kd}", M, 768, Kd, True, True)
for Kd in (64, 768):
    run(f"N3072 K{Kd}", M, 3072, Kd, True, True)
run("N768 K768 f32out", M, 768, 768, False, True)
