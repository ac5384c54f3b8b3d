"""conv0 GroupNorm forward / backward timings at the distill-step shape (B = 16 x 10 s, C = 512), every
DPH_C0B_VARIANT of the backward (read once per process: pass the variant as argv[1]).
usage: python tools/conv0_bench.py [variant] [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
if len(sys.argv) > 1:
    os.environ["DPH_C0B_VARIANT"] = sys.argv[1]
from dphubert_amd import _lib  # noqa: E402
from dphubert_amd._lib import call, ptr  # noqa: E402

B, S, C = 16, 160000, 512
L0 = (S - 10) // 5 + 1
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = "cuda"
s = _lib.stream_ptr()
wave = torch.randn(B, S, device=dev) * 0.1
w = torch.randn(C, 10, device=dev) * 0.3
gamma = torch.rand(C, device=dev) + 0.5
beta = torch.randn(C, device=dev) * 0.1
mask = torch.rand(C, device=dev)
y = torch.empty(B, L0, C, device=dev, dtype=torch.bfloat16)
mean = torch.empty(B * C, device=dev)
rstd = torch.empty(B * C, device=dev)
ws_f = torch.empty(B * 16 * 65 * 2, device=dev)
dy = (torch.randn(B, L0, C, device=dev) * 0.01).to(torch.bfloat16)
wsb = torch.empty(_lib.lib().dph_conv0_gn_bwd_workspace(B, S, C) // 4 + 64, device=dev)
dw = torch.zeros(C, 10, device=dev)
dg, db, dm = (torch.zeros(C, device=dev) for _ in range(3))


def fwd():
    call("dph_conv0_gn_fwd", ptr(wave), B, S, ptr(w), C, 10, 5, ptr(gamma), ptr(beta), ptr(mask), ptr(y), ptr(mean),
         ptr(rstd), ptr(ws_f), ws_f.numel() * 4, s)


def bwd():
    call("dph_conv0_gn_bwd", ptr(wave), B, S, ptr(w), C, 10, 5, ptr(gamma), ptr(beta), ptr(mask), ptr(mean),
         ptr(rstd), ptr(dy), ptr(dw), ptr(dg), ptr(db), ptr(dm), ptr(wsb), wsb.numel() * 4, s)


def timeit(f):
    f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


fwd()
tf, tb = timeit(fwd), timeit(bwd)
dyb = B * L0 * C * 2
print(f"variant {os.environ.get('DPH_C0B_VARIANT', '0')}: fwd {tf:7.1f} us  bwd {tb:7.1f} us "
      f"({dyb / tb / 1e3:6.0f} GB/s on the {dyb / 1e6:.0f} MB dy stream)", flush=True)
