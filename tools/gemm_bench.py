"""GEMM microbenchmark on the shapes of the HuBERT-Base distill step (B=16 x 10 s)."""
import sys
import time

import torch

sys.path.insert(0, ".")
from dphubert_amd import kernels as K  # noqa: E402

M = 16 * 499
SHAPES = [  # (name, M, N, K, a_kcontig, b_kcontig)
    ("qkv fwd", M, 2304, 768, True, True),
    ("ffn1 fwd+gelu", M, 3072, 768, True, True),
    ("ffn2 fwd", M, 768, 3072, True, True),
    ("oproj fwd", M, 768, 768, True, True),
    ("conv1 fwd", 16 * 15999, 512, 1536, True, True),
    ("conv1 dgrad", 16 * 15999, 1536, 512, True, False),
    ("conv1 wgrad", 512, 1536, 16 * 15999, False, False),
    ("ffn2 dgrad", M, 3072, 768, True, False),
    ("ffn1 dgrad", M, 768, 3072, True, False),
    ("qkv dgrad", M, 768, 2304, True, False),
    ("ffn1 dgrad kk", M, 768, 3072, True, True),
    ("qkv dgrad kk", M, 768, 2304, True, True),
    ("ffn1 wgrad", 3072, 768, M, False, False),
    ("qkv wgrad", 2304, 768, M, False, False),
    ("sq 4096", 4096, 4096, 4096, True, True),
    ("sq 8192", 8192, 8192, 8192, True, True),
]


def run(name, M, N, Kd, ak, bk, iters=20):
    A = (torch.randn(M, Kd, device="cuda") if ak else torch.randn(Kd, M, device="cuda")).to(torch.bfloat16)
    B = (torch.randn(N, Kd, device="cuda") if bk else torch.randn(Kd, N, device="cuda")).to(torch.bfloat16)
    out_f32 = not ak
    C = torch.empty(M, N, device="cuda", dtype=torch.float32 if out_f32 else torch.bfloat16)
    splits = K.choose_splits(M, N, Kd) if not ak else 1
    act = K.ACT_GELU if "gelu" in name else K.ACT_NONE

    def f():
        return K.gemm(K.dense(A), K.dense(B), K.dense(C), M, N, Kd, a_kcontig=ak, b_kcontig=bk,
                      c_dtype=K.OUT_F32 if out_f32 else K.OUT_BF16, splits=splits, act=act)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        ws = f()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    tf = 2 * M * N * Kd / ms / 1e9
    # library reference point: torch.matmul (hipBLASLt) on the same operands, plain bf16 output
    At = A if ak else A.t()
    Bt = B.t() if bk else B
    for _ in range(3):
        torch.matmul(At, Bt)
    e0.record()
    for _ in range(iters):
        torch.matmul(At, Bt)
    e1.record()
    torch.cuda.synchronize()
    ms_lib = e0.elapsed_time(e1) / iters
    print(f"{name:16s} M={M:6d} N={N:5d} K={Kd:5d} splits={splits:2d}  {ms*1e3:8.1f} us  {tf:6.0f} TF/s   "
          f"torch.matmul {ms_lib*1e3:8.1f} us {2 * M * N * Kd / ms_lib / 1e9:6.0f} TF/s", flush=True)
    return ms


if __name__ == "__main__":
    tot = 0.0
    for s in SHAPES:
        tot += run(*s)
    print(f"sum {tot*1e3:.1f} us")
