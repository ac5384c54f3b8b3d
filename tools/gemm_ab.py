"""A/B of GEMM paths (DPH_GEMM_PATH values) on the step's k-contiguous shapes, interleaved rounds in one
process, each path's output checked against the default path's.

    python tools/gemm_ab.py [path ...]        (default: auto pp256 pp128x256 pp256x128 pp128x192 pp128)
"""
import os
import sys

import torch

sys.path.insert(0, ".")
from dphubert_amd import kernels as K  # noqa: E402

M = 16 * 499
SHAPES = [  # (name, M, N, K, act); GELU_BWD: aux_in = a pre-activation, colmask, column sums (the FFN dgrad)
    ("qkv fwd", M, 2304, 768, K.ACT_NONE),
    ("ffn1 fwd+gelu", M, 3072, 768, K.ACT_GELU),
    ("ffn2 fwd", M, 768, 3072, K.ACT_NONE),
    ("oproj fwd", M, 768, 768, K.ACT_NONE),
    ("ffn2 dgrad kk", M, 3072, 768, K.ACT_NONE),
    ("ffn2 dgrad gelu'", M, 3072, 768, K.ACT_GELU_BWD),
    ("ffn1 dgrad kk", M, 768, 3072, K.ACT_NONE),
    ("qkv dgrad kk", M, 768, 2304, K.ACT_NONE),
    ("conv1 fwd", 16 * 15999, 512, 1536, K.ACT_NONE),
    ("conv2 fwd", 16 * 7999, 512, 1536, K.ACT_NONE),
    ("sq 4096", 4096, 4096, 4096, K.ACT_NONE),
    ("sq 8192", 8192, 8192, 8192, K.ACT_NONE),
]


def main():
    paths = sys.argv[1:] or ["auto", "pp256", "pp128x256", "pp256x128", "pp128x192", "pp128"]
    rounds, iters = 3, 10
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, m, n, k, act in SHAPES:
        A = (torch.rand(m, k, device="cuda") * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(n, k, device="cuda") * 2 - 1).to(torch.bfloat16)
        bias = torch.randn(n, device="cuda")
        outs = {p: torch.empty(m, n, device="cuda", dtype=torch.bfloat16) for p in paths}
        times = {p: [] for p in paths}

        kw = dict(bias=bias)
        if act == K.ACT_GELU_BWD:
            kw = dict(aux_in=(torch.randn(m, n, device="cuda")).to(torch.bfloat16),
                      colmask=(torch.rand(n, device="cuda") > 0.2).float(), colsum_out=torch.zeros(n, device="cuda"),
                      colsum_aux=torch.zeros(n, device="cuda"))

        def f(p):
            if p == "auto":
                os.environ.pop("DPH_GEMM_PATH", None)
            else:
                os.environ["DPH_GEMM_PATH"] = p
            K.gemm(K.dense(A), K.dense(B), K.dense(outs[p]), m, n, k, a_kcontig=True, b_kcontig=True,
                   c_dtype=K.OUT_BF16, act=act, **kw)
        for p in paths:
            f(p)
        torch.cuda.synchronize()
        for _ in range(rounds):
            for p in paths:
                e0.record()
                for _ in range(iters):
                    f(p)
                e1.record()
                torch.cuda.synchronize()
                times[p].append(e0.elapsed_time(e1) / iters)
        os.environ.pop("DPH_GEMM_PATH", None)
        ref = outs[paths[0]].float()
        row = f"{name:14s} {m:6d}x{n:5d}x{k:5d} "
        for p in paths:
            ms = min(times[p])
            err = ((outs[p].float() - ref).norm() / ref.norm()).item()
            row += f"| {p} {ms * 1e3:7.1f} us {2 * m * n * k / ms / 1e9:5.0f} TF e={err:.1e} "
        print(row, flush=True)
        del A, B, outs


if __name__ == "__main__":
    main()
