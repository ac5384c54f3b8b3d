"""Sweep of the ppw weight-gradient kernel over (tile, split-K) on the step's wgrad shapes (DPH_PPW_FORCE),
against the register-staged kernel (DPH_GEMM_PPW=0) with its own split heuristic.  Data for ppw_plan.

    python tools/wgrad_sweep.py
"""
import os
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from dphubert_amd import kernels as K  # noqa: E402
from wgrad_ab import SHAPES, B  # noqa: E402

KINDS = {12: "256x256", 15: "128x192", 13: "128x256", 16: "128x128"}
SPLITS = [1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 21, 24, 32]


def main():
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for name, n, kin, frames, conv in SHAPES:
        dy = (torch.randn(frames, n, device="cuda") * 0.5).to(torch.bfloat16)
        if conv is None:
            x = (torch.randn(frames, kin, device="cuda") * 0.5).to(torch.bfloat16)
            Bm = K.dense(x)
        else:
            lin, k, s = conv
            C = kin // k
            x = (torch.randn(B, lin, C, device="cuda") * 0.5).to(torch.bfloat16)
            Bm = K.mat(x, row_stride=s * C, rows_per_batch=frames // B, batch_stride=lin * C)
        out = torch.zeros(n, kin, device="cuda")
        res = []

        def run(env, splits, iters=8):
            for k_ in ("DPH_GEMM_PPW", "DPH_PPW_FORCE"):
                os.environ.pop(k_, None)
            os.environ.update(env)
            keep = [K.gemm(K.dense(dy), Bm, K.dense(out), n, kin, frames, a_kcontig=False, b_kcontig=False,
                           c_dtype=K.OUT_F32, splits=splits)]
            torch.cuda.synchronize()
            e0.record()
            for _ in range(iters):
                keep.append(K.gemm(K.dense(dy), Bm, K.dense(out), n, kin, frames, a_kcontig=False,
                                   b_kcontig=False, c_dtype=K.OUT_F32, splits=splits))
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / iters * 1e3
        os.environ["DPH_GEMM_PPW"] = "0"
        s_old = K.choose_splits(n, kin, frames)
        t_old = min(run({"DPH_GEMM_PPW": "0"}, s_old) for _ in range(2))
        for kind in KINDS:
            for sp in SPLITS:
                os.environ.pop("DPH_GEMM_PPW", None)
                os.environ["DPH_PPW_FORCE"] = f"{kind}:{sp}"
                got = K.choose_splits(n, kin, frames)
                if got != sp:
                    continue
                t = min(run({"DPH_PPW_FORCE": f"{kind}:{sp}"}, sp) for _ in range(2))
                res.append((t, KINDS[kind], sp))
        for k_ in ("DPH_GEMM_PPW", "DPH_PPW_FORCE"):
            os.environ.pop(k_, None)
        s_plan = K.choose_splits(n, kin, frames)
        t_plan = run({}, s_plan)
        res.sort()
        best = " ".join(f"{nm}/s{sp}:{t:.1f}" for t, nm, sp in res[:6])
        print(f"{name:12s} old s={s_old:2d} {t_old:7.1f} us | plan s={s_plan:2d} {t_plan:7.1f} us | best {best}",
              flush=True)


if __name__ == "__main__":
    main()
