"""Fixed (K-independent) cost of a ping-pong GEMM launch: M = 7984, N = 768 projections at K = 128 .. 3072, timed as
20 launches captured in one HIP graph (the step's regime), plus a 1-element kernel for the graph's per-launch floor.
usage: python tools/gemm_fixed.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dphubert_amd import _lib, kernels as K  # noqa: E402
from dphubert_amd._lib import call, ptr  # noqa: E402

M = 7984
dev = "cuda"


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


z = torch.zeros(64, device=dev)
print(f"1-element kernel in a graph: {graph_time(lambda: call('dph_cast_bf16', ptr(z), ptr(z), 1, _lib.stream_ptr())):6.2f} us",
      flush=True)
for N in (768, 2304):
    for Kd in (128, 256, 512, 768, 1536, 3072):
        A = (torch.rand(M, Kd, device=dev) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(N, Kd, device=dev) * 2 - 1).to(torch.bfloat16)
        Cm = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        t = graph_time(lambda: K.gemm(K.dense(A), K.dense(B), K.dense(Cm), M, N, Kd, a_kcontig=True, b_kcontig=True))
        print(f"M={M} N={N} K={Kd:5d}: {t:7.2f} us  ({2.0 * M * N * Kd / t / 1e6:6.0f} TF/s)", flush=True)
