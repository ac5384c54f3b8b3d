"""Microbench of dph_conv0_gn_bwd at the bench shape (16 x 10 s utterances, C=512).
Variant via DPH_C0B_VARIANT (read once per process).  Run on the GPU box."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from test_ops_gpu import _conv0_gn  # noqa: E402


def main():
    B, S, C = 16, 160000, 512
    g = torch.Generator().manual_seed(0)
    wave = (0.1 * torch.randn(B, S, generator=g)).cuda()
    w = torch.randn(C, 10, generator=g).cuda()
    gamma, beta, mask = torch.ones(C).cuda(), torch.zeros(C).cuda(), torch.rand(C, generator=g).cuda()
    L0 = (S - 10) // 5 + 1
    dy = torch.randn(B, L0, C, device="cuda").to(torch.bfloat16)
    for _ in range(3):
        _conv0_gn(wave, w, C, gamma, beta, mask, dy)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 20
    for _ in range(n):
        _conv0_gn(wave, w, C, gamma, beta, mask, dy)
    e1.record()
    torch.cuda.synchronize()
    print(f"variant {os.environ.get('DPH_C0B_VARIANT', '0')}: fwd+bwd {e0.elapsed_time(e1) / n * 1e3:.1f} us")


if __name__ == "__main__":
    main()
