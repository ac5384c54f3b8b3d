"""Bitwise run-to-run determinism of the forward kernels (a race shows up as a mismatch)."""
import sys

import torch

sys.path.insert(0, ".")
from dphubert_amd import _lib  # noqa: E402
from dphubert_amd import kernels as K  # noqa: E402
from dphubert_amd._lib import call, ptr  # noqa: E402

DEV = "cuda"
s = _lib.stream_ptr()


def check(name, fn, n=20):
    ref = [t.clone() for t in fn()]
    bad = 0
    worst = 0.0
    for _ in range(n):
        out = fn()
        for a, b in zip(ref, out):
            if not torch.equal(a, b):
                bad += 1
                worst = max(worst, (a.float() - b.float()).abs().max().item())
    torch.cuda.synchronize()
    print(f"{name:40s} mismatching runs {bad}/{n}  worst |diff| {worst:.3g}", flush=True)


torch.manual_seed(0)
for (B, T, H) in [(2, 99, 12), (4, 499, 12), (2, 1999, 12)]:
    D = H * 64
    M = B * T
    qkv = (torch.randn(M, 3 * D, device=DEV) * 2).to(torch.bfloat16)
    hm = torch.rand(H, device=DEV)
    lens = torch.full((B,), T, device=DEV, dtype=torch.int64)

    def att():
        o_u = torch.empty(M, D, device=DEV, dtype=torch.float32)
        o_m = torch.empty(o_u.shape, device=o_u.device, dtype=torch.bfloat16)
        lse = torch.empty(B * H * T, device=DEV)
        call("dph_attention_fwd", ptr(qkv), ptr(o_u), ptr(o_m), ptr(lse), ptr(hm), ptr(lens), B, T, H, 0.125, 0.0, 0, None,
             s)
        return o_u, o_m, lse

    check(f"attention_fwd B{B} T{T}", att)
    g = torch.randn(M, D, device=DEV).to(torch.bfloat16)
    o_u, o_m, lse = att()

    def attb():
        Dv = torch.empty(B * H * T, device=DEV)
        dhm = torch.zeros(H, device=DEV)
        call("dph_attention_bwd_prep", ptr(g), ptr(o_u), ptr(hm), ptr(Dv), ptr(dhm), B, T, H, s)
        dqkv = torch.empty_like(qkv)
        call("dph_attention_bwd", ptr(qkv), ptr(g), ptr(hm), ptr(lse), ptr(Dv), ptr(dqkv), ptr(lens), B, T, H, 0.125,
             0.0, 0, None, s)
        return (dqkv,)

    check(f"attention_bwd B{B} T{T}", attb)
    x = torch.randn(M, D, device=DEV).to(torch.bfloat16)
    w = (torch.randn(3072, D, device=DEV) * 0.05).to(torch.bfloat16)
    b = torch.randn(3072, device=DEV)
    check(f"gemm gelu fwd M{M}", lambda: (K.linear_fwd(x, w, b, act=K.ACT_GELU),))
    w2 = (torch.randn(D, 3072, device=DEV) * 0.05).to(torch.bfloat16)
    f = K.linear_fwd(x, w, b, act=K.ACT_GELU)
    check(f"gemm resid fwd M{M}", lambda: (K.linear_fwd(f, w2, None, residual=x),))
    lw = torch.rand(D, device=DEV)
    lb = torch.rand(D, device=DEV)

    def ln():
        y = torch.empty_like(x)
        mu = torch.empty(M, device=DEV)
        rs = torch.empty(M, device=DEV)
        call("dph_layernorm_fwd", ptr(x), None, ptr(lw), ptr(lb), ptr(y), ptr(mu), ptr(rs), M, D, 1e-5, 0.0, 0, s)
        return y, mu, rs

    check(f"layernorm_fwd M{M}", ln)

# ring GEMM shapes of the Large family (persistent 128 x 256 tiles), with and without row-length zeroing
for (M, N, Kd) in [(998, 1024, 1024), (998, 1024, 4096), (998, 4096, 1024), (7984, 768, 3072), (7984, 3072, 768)]:
    x = (torch.randn(M, Kd, device=DEV) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, Kd, device=DEV) * 0.05).to(torch.bfloat16)
    b = torch.randn(N, device=DEV)
    r = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    rl = torch.tensor([M // 2 - 7, M // 2], device=DEV, dtype=torch.int64)
    check(f"gemm {M}x{N}x{Kd} resid", lambda: (K.linear_fwd(x, w, b, residual=r),))
    check(f"gemm {M}x{N}x{Kd} gelu rowlen", lambda: (K.linear_fwd(x, w, b, act=K.ACT_GELU, row_len=rl, len_rows=M // 2),))
