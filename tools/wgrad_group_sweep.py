"""Sweep of the grouped weight-gradient launch (dph_gemm_grouped: n encoder layers' dW = dY^T X of one shape in one
launch) over (tile, split-K) via DPH_PPW_FORCE, against the plan's own choice.  Data for ppw_plan at batch > 1.

    python tools/wgrad_group_sweep.py [n]
"""
import os
import sys

import torch

sys.path.insert(0, ".")
from dphubert_amd import kernels as K  # noqa: E402

FRAMES = 7984
SHAPES = [("qkv", 2304, 768), ("oproj", 768, 768), ("ffn1", 3072, 768), ("ffn2", 768, 3072)]
KINDS = {12: "256x256", 15: "128x192", 13: "128x256", 16: "128x128"}
SPLITS = [1, 2, 3, 4, 6]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, N, Kin in SHAPES:
        items = [((torch.randn(FRAMES, N, device="cuda") * 0.5).to(torch.bfloat16),
                  (torch.randn(FRAMES, Kin, device="cuda") * 0.5).to(torch.bfloat16),
                  torch.zeros(N, Kin, device="cuda")) for _ in range(n)]
        flop = 2.0 * FRAMES * N * Kin * n

        def run(iters=6):
            keep = [K.linear_wgrad_grouped(items)]
            torch.cuda.synchronize()
            e0.record()
            for _ in range(iters):
                keep.append(K.linear_wgrad_grouped(items))
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / iters * 1e3

        os.environ.pop("DPH_PPW_FORCE", None)
        s_plan = K.choose_splits(N, Kin, FRAMES, batch=n)
        t_plan = min(run() for _ in range(2))
        res = []
        for kind in KINDS:
            for sp in SPLITS:
                os.environ["DPH_PPW_FORCE"] = f"{kind}:{sp}"
                if K.choose_splits(N, Kin, FRAMES, batch=n) != sp:
                    continue
                res.append((min(run() for _ in range(2)), KINDS[kind], sp))
        os.environ.pop("DPH_PPW_FORCE", None)
        res.sort()
        best = " ".join(f"{k}/s{s} {t:.1f}us" for t, k, s in res[:4])
        print(f"{name:6s} n={n} {N}x{Kin}x{FRAMES}: plan s={s_plan} {t_plan:.1f} us {flop / t_plan / 1e6:.0f} TF | "
              f"best: {best} ({flop / res[0][0] / 1e6:.0f} TF)", flush=True)


if __name__ == "__main__":
    main()
