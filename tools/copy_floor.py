"""Floor of a one-round memory-bound launch at the LayerNorm shapes: torch copy of a 7984 x 768 bf16 tensor (12 MB
in + 12 MB out) and of fp32 rows, and the LayerNorm forward / backward of the same rows, each 20x in one HIP graph.
usage: python tools/copy_floor.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dphubert_amd import _lib  # noqa: E402
from dphubert_amd._lib import call, ptr  # noqa: E402


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


M, D = 7984, 768
x = torch.randn(M, D, device="cuda").to(torch.bfloat16)
y = torch.empty_like(x)
x2 = torch.randn(2 * M, D, device="cuda").to(torch.bfloat16)
y2 = torch.empty_like(x2)
w = torch.rand(D, device="cuda") + 0.5
b = torch.randn(D, device="cuda")
mu = torch.empty(M, device="cuda")
rs = torch.empty(M, device="cuda")
dy = torch.randn(M, D, device="cuda").to(torch.bfloat16)
dx = torch.empty_like(x)
br = torch.empty_like(x)
pre = torch.randn(M, D, device="cuda").to(torch.bfloat16)
dg, db, bcs, sd = (torch.zeros(D, device="cuda") for _ in range(4))
sm = torch.ones(1, device="cuda")
wsb = torch.empty(_lib.lib().dph_layernorm_bwd_workspace(M, D) // 4, device="cuda")
call("dph_layernorm_fwd", ptr(x), None, ptr(w), ptr(b), ptr(y), ptr(mu), ptr(rs), M, D, 1e-5, 0.0, 0, _lib.stream_ptr())


def ln_bwd():
    call("dph_layernorm_bwd", ptr(dy), ptr(x), None, ptr(w), ptr(mu), ptr(rs), ptr(dx), ptr(dg), ptr(db), M, D, 0.0, 0,
         ptr(br), 0.1, 7, None, ptr(bcs), None, None, ptr(wsb), wsb.numel() * 4, _lib.stream_ptr())


def ln_bwd_lm():
    call("dph_layernorm_bwd", ptr(dy), ptr(x), None, ptr(w), ptr(mu), ptr(rs), ptr(dx), ptr(dg), ptr(db), M, D, 0.0, 0,
         ptr(br), 0.1, 7, ptr(sm), ptr(bcs), ptr(pre), ptr(sd), ptr(wsb), wsb.numel() * 4, _lib.stream_ptr())


def ln_bwd_plain():
    call("dph_layernorm_bwd", ptr(dy), ptr(x), None, ptr(w), ptr(mu), ptr(rs), ptr(dx), ptr(dg), ptr(db), M, D, 0.0, 0,
         None, 0.0, 0, None, None, None, None, ptr(wsb), wsb.numel() * 4, _lib.stream_ptr())


def ln_bwd_p0():
    call("dph_layernorm_bwd", ptr(dy), ptr(x), None, ptr(w), ptr(mu), ptr(rs), ptr(dx), ptr(dg), ptr(db), M, D, 0.0, 0,
         ptr(br), 0.0, 7, None, ptr(bcs), None, None, ptr(wsb), wsb.numel() * 4, _lib.stream_ptr())


def ln_bwd_nocol():
    call("dph_layernorm_bwd", ptr(dy), ptr(x), None, ptr(w), ptr(mu), ptr(rs), ptr(dx), None, None, M, D, 0.0, 0,
         ptr(br), 0.1, 7, None, None, None, None, ptr(wsb), wsb.numel() * 4, _lib.stream_ptr())


for name, f, byt in (
        ("layernorm bwd plain", ln_bwd_plain, 3 * M * D * 2),
        ("layernorm bwd (+branch p=0)", ln_bwd_p0, 4 * M * D * 2),
        ("layernorm bwd (+branch, no colsums)", ln_bwd_nocol, 4 * M * D * 2),
        ("layernorm bwd (+branch)", ln_bwd, 5 * M * D * 2),
        ("layernorm bwd (+layer mask)", ln_bwd_lm, 6 * M * D * 2),
        ("copy bf16 12 MB -> 12 MB", lambda: y.copy_(x), 2 * M * D * 2),
        ("copy bf16 24 MB -> 24 MB", lambda: y2.copy_(x2), 2 * 2 * M * D * 2),
        ("layernorm fwd", lambda: call("dph_layernorm_fwd", ptr(x), None, ptr(w), ptr(b), ptr(y), ptr(mu), ptr(rs), M, D,
                                       1e-5, 0.0, 0, _lib.stream_ptr()), 2 * M * D * 2)):
    t = graph_time(f)
    print(f"{name:28s} {t:7.2f} us  {byt / t / 1e3:7.0f} GB/s", flush=True)
