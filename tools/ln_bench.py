"""LayerNorm fwd/bwd microbenchmark on the encoder shape (7984 x 768): variants of the backward."""
import sys

import torch

sys.path.insert(0, ".")
from dphubert_amd import ops  # noqa: E402
from dphubert_amd._lib import call, ptr  # noqa: E402

M, D = 7984, 768
dev = "cuda"
x = torch.randn(M, D, device=dev).to(torch.bfloat16)
dy = torch.randn(M, D, device=dev).to(torch.bfloat16)
w = torch.rand(D, device=dev) + 0.5
b = torch.randn(D, device=dev)
y = torch.empty_like(x)
mu = torch.empty(M, device=dev)
rs = torch.empty(M, device=dev)
dx = torch.empty_like(x)
br = torch.empty_like(x)
dw = torch.zeros(D, device=dev)
db = torch.zeros(D, device=dev)
dc = torch.zeros(D, device=dev)
s = ops._s()


def timeit(f, n=50):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


fwd = lambda: call("dph_layernorm_fwd", ptr(x), None, ptr(w), ptr(b), ptr(y), ptr(mu), ptr(rs), M, D, 1e-5, 0.0, 0, s)
print(f"fwd                      {timeit(fwd):7.1f} us  ({2 * M * D * 2 / timeit(fwd) / 1e3:.2f} TB/s)")
ws = ops.ln_ws(M, D, dev)
variants = {
    "bwd dx only": lambda: call("dph_layernorm_bwd", ptr(dy), ptr(x), None, ptr(w), ptr(mu), ptr(rs), ptr(dx), None,
                                None, M, D, 0.0, 0, None, 0.0, 0, None, None, None, None, *ws, s),
    "bwd +dgamma/dbeta": lambda: call("dph_layernorm_bwd", ptr(dy), ptr(x), None, ptr(w), ptr(mu), ptr(rs), ptr(dx),
                                      ptr(dw), ptr(db), M, D, 0.0, 0, None, 0.0, 0, None, None, None, None, *ws, s),
    "bwd +branch p=0": lambda: call("dph_layernorm_bwd", ptr(dy), ptr(x), None, ptr(w), ptr(mu), ptr(rs), ptr(dx),
                                    ptr(dw), ptr(db), M, D, 0.0, 0, ptr(br), 0.0, 0, None, ptr(dc), None, None, *ws, s),
    "bwd +branch p=0.1": lambda: call("dph_layernorm_bwd", ptr(dy), ptr(x), None, ptr(w), ptr(mu), ptr(rs), ptr(dx),
                                      ptr(dw), ptr(db), M, D, 0.0, 0, ptr(br), 0.1, 7, None, ptr(dc), None, None, *ws,
                                      s),
}
for k, f in variants.items():
    t = timeit(f)
    print(f"{k:24s} {t:7.1f} us")
