"""Run one GEMM shape a few times (for rocprofv3 counter collection).
usage: DPH_GEMM_PATH=big python tools/gemm_one.py M N K [iters]"""
import sys

import torch

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), ".."))
from dphubert_amd import kernels as K  # noqa: E402

M, N, Kd = (int(x) for x in sys.argv[1:4])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 5
A = (torch.rand(M, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
B = (torch.rand(N, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(iters):
    K.gemm(K.dense(A), K.dense(B), K.dense(C), M, N, Kd, a_kcontig=True, b_kcontig=True)
torch.cuda.synchronize()
