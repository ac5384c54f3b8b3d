"""In-process A/B of GEMM paths (DPH_GEMM_PATH is read per call) on the step's GEMM shapes: interleaved rounds,
median per (shape, path).  usage: python tools/gemm_variants.py [rounds] [path ...]  (default: auto mid mid8)"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dphubert_amd import kernels as K  # noqa: E402

M = 16 * 499
SHAPES = [("qkv fwd", M, 2304, 768), ("ffn1 fwd+gelu", M, 3072, 768), ("ffn2 fwd", M, 768, 3072),
          ("oproj fwd", M, 768, 768), ("ffn2 dgrad(T)", M, 3072, 768), ("ffn1 dgrad(T)", M, 768, 3072),
          ("qkv dgrad(T)", M, 768, 2304), ("conv2 fwd", 16 * 7999, 512, 1536), ("conv1 fwd", 16 * 15999, 512, 1536),
          ("conv1 dgrad", 16 * 15999, 1536, 512)]
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
paths = sys.argv[2:] or ["auto", "mid", "mid8"]
res = {}
data = {}
for name, m, n, k in SHAPES:
    A = (torch.rand(m, k, device="cuda") * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(n, k, device="cuda") * 2 - 1).to(torch.bfloat16)
    C = torch.empty(m, n, device="cuda", dtype=torch.bfloat16)
    bias = torch.randn(n, device="cuda")
    pre = torch.empty_like(C) if "gelu" in name else None
    data[name] = (A, B, C, bias, pre, m, n, k)


def run(name, path, iters=20):
    A, B, C, bias, pre, m, n, k = data[name]
    os.environ.pop("DPH_GEMM_PERSIST", None)
    if path.endswith("-np"):                 # one tile per block (no persistent grid)
        os.environ["DPH_GEMM_PERSIST"] = "0"
        path = path[:-3]
    if path == "auto":
        os.environ.pop("DPH_GEMM_PATH", None)
    else:
        os.environ["DPH_GEMM_PATH"] = path
    act = K.ACT_GELU if pre is not None else K.ACT_NONE
    f = lambda: K.gemm(K.dense(A), K.dense(B), K.dense(C), m, n, k, a_kcontig=True, b_kcontig=True,  # noqa: E731
                       bias=bias, act=act, pre_out=pre)
    for _ in range(2):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


for r in range(rounds):
    for name, *_ in SHAPES:
        for p in paths:
            res.setdefault((name, p), []).append(run(name, p))
os.environ.pop("DPH_GEMM_PATH", None)
os.environ.pop("DPH_GEMM_PERSIST", None)
for name, m, n, k in SHAPES:
    row = []
    for p in paths:
        t = statistics.median(res[(name, p)])
        row.append(f"{p} {t:7.1f} us {2 * m * n * k / t / 1e6:5.0f} TF/s")
    print(f"{name:15s} {m}x{n}x{k}: " + " | ".join(row), flush=True)
