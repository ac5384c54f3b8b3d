"""Attention kernel timings on the distill-step shape (B=16, T=499, H=12, hd=64), dropout 0 / 0.1."""
import sys

import torch

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)),
                                              ".."))
from dphubert_amd import _lib  # noqa: E402
from dphubert_amd._lib import call, ptr  # noqa: E402
from dphubert_amd.ops import _ws  # noqa: E402


def prep_ws(B, T, H):
    return _ws(_lib.lib().dph_attention_bwd_prep_workspace(B, T, H), "cuda")

B, T, H = 16, 499, 12
D = H * 64
M = B * T
s = _lib.stream_ptr()
qkv = (torch.randn(M, 3 * D, device="cuda") * 0.5).to(torch.bfloat16)
hm = torch.rand(H, device="cuda")
lens = torch.full((B,), T, device="cuda", dtype=torch.int64)
o_u = torch.empty(M, D, device="cuda", dtype=torch.float32)
o_m = torch.empty(o_u.shape, device=o_u.device, dtype=torch.bfloat16)
lse = torch.empty(B * H * T, device="cuda")
g = torch.randn(M, D, device="cuda").to(torch.bfloat16)
Dv = torch.empty(B * H * T, device="cuda")
dhm = torch.zeros(H, device="cuda")
dqkv = torch.empty_like(qkv)


def timeit(f, n=20):
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


keep = torch.empty(_lib.lib().dph_attention_keep_bytes(B, T, H) // 8, dtype=torch.int64, device="cuda")
for p, kb in ((0.0, None), (0.1, None), (0.1, keep)):
    fwd = lambda: call("dph_attention_fwd", ptr(qkv), ptr(o_u), ptr(o_m), ptr(lse), ptr(hm), ptr(lens), B, T, H,  # noqa
                       0.125, p, 7, ptr(kb), s)
    prep = lambda: call("dph_attention_bwd_prep", ptr(g), ptr(o_u), ptr(hm), ptr(Dv), ptr(dhm), B, T, H, *prep_ws(B, T, H), s)  # noqa
    bwd = lambda: call("dph_attention_bwd", ptr(qkv), ptr(g), ptr(hm), ptr(lse), ptr(Dv), ptr(dqkv), ptr(lens),  # noqa
                       B, T, H, 0.125, p, 7, ptr(kb), s)
    tf, tp, tb = timeit(fwd), timeit(prep), timeit(bwd)
    fl = 4.0 * B * H * T * T * 64
    print(f"p={p}{' keep-bits' if kb is not None else ''}: fwd {tf:7.1f} us ({fl / tf / 1e6:5.0f} TF/s)  prep {tp:6.1f} us  bwd {tb:7.1f} us "
          f"({2.5 * fl / tb / 1e6:5.0f} TF/s)", flush=True)
