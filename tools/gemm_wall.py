"""Wall time of the step's main ping-pong GEMM shapes (20 launches captured in one HIP graph, best of 5 replays), for
library A/B (DPH_LIB_PATH) and tile / schedule switches (DPH_PP_FORCE, DPH_PP_RING3).

    python tools/gemm_wall.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dphubert_amd import kernels as K  # noqa: E402

SHAPES = [  # M, N, K, epilogue (resid: bf16 residual add), what it is in the step
    (7984, 768, 3072, True, "FFN2 fwd / FFN1 dgrad"),
    (7984, 768, 2304, True, "QKV dgrad"),
    (7984, 768, 768, True, "out-proj fwd / dgrad"),
    (7984, 2304, 768, False, "QKV fwd"),
    (7984, 3072, 768, False, "FFN1 fwd (plain)"),
    (255984, 512, 1536, False, "conv1 fwd"),
    (7984, 3072, 768, "gelu", "FFN1 fwd, GELU + stored factor + dropout (student)"),
    (7984, 3072, 768, "gelu0", "FFN1 fwd, GELU (teacher)"),
]


def graph_time(f, n=20, reps=5):
    f()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                f()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / n * 1e3)
    return best


for M, N, Kd, resid, what in SHAPES:
    A = (torch.rand(M, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    R = torch.randn(M, N, device="cuda").to(torch.bfloat16) if resid is True else None
    kw = {}
    if resid in ("gelu", "gelu0"):
        bias = torch.randn(N, device="cuda") * 0.1
        kw = dict(act=K.ACT_GELU, bias=bias)
        if resid == "gelu":
            U = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            kw.update(pre_out=U, dropout_p=0.1, seed=5, colmask=torch.rand(N, device="cuda"),
                      flags=K.GEMM_PRE_DGK)
    f = lambda: K.gemm(K.dense(A), K.dense(B), K.dense(C), M, N, Kd, a_kcontig=True, b_kcontig=True,  # noqa: E731
                       residual=R, **kw)
    t = graph_time(f)
    print(f"{M:6d} x {N:4d} x {Kd:4d}{' +res' if resid is True else '     '} {t:8.2f} us  {2 * M * N * Kd / t / 1e6:6.0f} TF/s  "
          f"{what}", flush=True)
    del A, B, C, R
