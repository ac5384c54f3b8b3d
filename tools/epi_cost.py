"""Epilogue feature cost on one GEMM shape: plain / +residual / +pre_out / +dropout / GELU combinations,
median of interleaved rounds.  usage: python tools/epi_cost.py [M N K] (default 7984 768 768)"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dphubert_amd import kernels as K  # noqa: E402

M, N, Kd = (int(x) for x in sys.argv[1:4]) if len(sys.argv) >= 4 else (7984, 768, 768)
A = (torch.rand(M, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
B = (torch.rand(N, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
R = torch.randn(M, N, device="cuda").to(torch.bfloat16)
P = torch.empty_like(C)
bias = torch.randn(N, device="cuda")
VARIANTS = {
    "plain": {},
    "res": dict(residual=R),
    "res+pre": dict(residual=R, pre_out=P),
    "res+pre+drop": dict(residual=R, pre_out=P, dropout_p=0.1, seed=5),
    "drop": dict(dropout_p=0.1, seed=5),
    "gelu": dict(act=K.ACT_GELU),
    "gelu+pre": dict(act=K.ACT_GELU, pre_out=P),
}


def run(kw, iters=20):
    f = lambda: K.gemm(K.dense(A), K.dense(B), K.dense(C), M, N, Kd, a_kcontig=True, b_kcontig=True,  # noqa: E731
                       bias=bias, **kw)
    for _ in range(2):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


paths = (os.environ.get("PATHS") or "auto").split(",")
res = {}
for r in range(5):
    for p in paths:
        if p == "auto":
            os.environ.pop("DPH_GEMM_PATH", None)
        else:
            os.environ["DPH_GEMM_PATH"] = p
        for name, kw in VARIANTS.items():
            res.setdefault((p, name), []).append(run(kw))
os.environ.pop("DPH_GEMM_PATH", None)
for p in paths:
    print(f"{M}x{N}x{Kd} path {p}: " + " | ".join(f"{n} {statistics.median(res[(p, n)]):6.1f}" for n in VARIANTS), flush=True)
