"""The (mn, mn) weight-gradient kernel (ppw_gemm_kernel: both operands [K][M] / [K][N], fragments by transposed LDS
reads) against the (k, k) ping-pong kernel (pp_gemm_kernel: both operands k-contiguous, ds_read_b128 fragments) on
the same math: C[M][N] (fp32) = A^T B over a long K, dense operands, 20 launches per HIP graph, median of 5.

    python tools/ppw_vs_pp.py [M N K]...
"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from dphubert_amd import kernels as K  # noqa: E402


def timed(f, iters=20, rounds=5):
    f()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(iters):
            f()
    res = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / iters * 1e3)
    return statistics.median(res)


def main():
    shapes = [(512, 1536, 255984), (2304, 768, 7984), (4096, 4096, 8192)]
    a = sys.argv[1:]
    if a:
        shapes = [tuple(int(x) for x in a[i:i + 3]) for i in range(0, len(a), 3)]
    for M, N, Kd in shapes:
        at = (torch.rand(Kd, M, device="cuda") * 2 - 1).to(torch.bfloat16)     # [K][M]
        bt = (torch.rand(Kd, N, device="cuda") * 2 - 1).to(torch.bfloat16)     # [K][N]
        ak = at.t().contiguous()                                                 # [M][K]
        bk = bt.t().contiguous()                                                 # [N][K]
        c = torch.zeros(M, N, device="cuda")
        fl = 2.0 * M * N * Kd
        keep = []

        def mn():
            keep.append(K.linear_wgrad(at, bt, c, accumulate=False))   # dW[M][N] = A^T B, ppw plan
            keep.clear()

        def kk():
            K.gemm(K.dense(ak), K.dense(bk), K.dense(c), M, N, Kd, a_kcontig=True, b_kcontig=True,
                   c_dtype=K.OUT_F32)
        t_mn, t_kk = timed(mn), timed(kk)
        print(f"{M}x{N}x{Kd}: (mn, mn) ppw {t_mn:8.1f} us = {fl / t_mn / 1e6:6.0f} TF/s | (k, k) pp {t_kk:8.1f} us = "
              f"{fl / t_kk / 1e6:6.0f} TF/s  [{K._variant_name(M, N, Kd) if hasattr(K, '_variant_name') else ''}]")


if __name__ == "__main__":
    main()
