"""A/B of the ppw tile order over (z, tile) (DPH_PPW_ZMAP=1, default) against the per-z-plane order (=0): the
grouped encoder-layer weight gradients (n = 12 layers per launch) and the split-K conv weight gradients of the
HuBERT-Base step, interleaved rounds in one process, outputs checked against each other.

    python tools/zmap_ab.py
"""
import os
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tools")
from dphubert_amd import kernels as K  # noqa: E402
from wgrad_ab import SHAPES, B  # noqa: E402

GROUPED = [("qkv x12", 2304, 768), ("oproj x12", 768, 768), ("ffn1 x12", 3072, 768), ("ffn2 x12", 768, 3072)]
FRAMES = 7984


def main():
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    cases = []
    for name, N, Kin in GROUPED:
        items = [((torch.randn(FRAMES, N, device="cuda") * 0.5).to(torch.bfloat16),
                  (torch.randn(FRAMES, Kin, device="cuda") * 0.5).to(torch.bfloat16),
                  torch.zeros(N, Kin, device="cuda")) for _ in range(12)]
        cases.append((name, lambda items=items: K.linear_wgrad_grouped(items, accumulate=False),
                      lambda items=items: torch.cat([dw.flatten() for _, _, dw in items])))
    for name, n, kin, frames, conv in SHAPES:
        if conv is None:
            continue
        lin, k, s = conv
        C = kin // k
        dy = (torch.randn(frames, n, device="cuda") * 0.5).to(torch.bfloat16)
        x = (torch.randn(B, lin, C, device="cuda") * 0.5).to(torch.bfloat16)
        out = torch.zeros(n, kin, device="cuda")
        sp = K.choose_splits(n, kin, frames)
        Bm = K.mat(x, row_stride=s * C, rows_per_batch=frames // B, batch_stride=lin * C)
        # (x rides along in the defaults: Bm holds only its raw pointer)
        cases.append((name, lambda dy=dy, x=x, Bm=Bm, out=out, n=n, kin=kin, frames=frames, sp=sp: K.gemm(
            K.dense(dy), Bm, K.dense(out), n, kin, frames, a_kcontig=False, b_kcontig=False, c_dtype=K.OUT_F32,
            splits=sp), lambda out=out: out.clone()))
    tot = {"0": 0.0, "1": 0.0}
    for name, fn, res in cases:
        t = {"0": [], "1": []}
        outs = {}
        for _ in range(3):
            for mode in ("0", "1"):
                os.environ["DPH_PPW_ZMAP"] = mode
                keep = [fn()]
                torch.cuda.synchronize()
                e0.record()
                for _ in range(8):
                    keep.append(fn())
                e1.record()
                torch.cuda.synchronize()
                t[mode].append(e0.elapsed_time(e1) / 8 * 1e3)
                outs[mode] = res()
        err = ((outs["0"] - outs["1"]).norm() / outs["0"].norm().clamp_min(1e-30)).item()
        a, b = min(t["0"]), min(t["1"])
        tot["0"] += a
        tot["1"] += b
        print(f"{name:12s} per-z {a:8.1f} us | zmap {b:8.1f} us | {100 * (a - b) / a:+5.1f} % | e={err:.1e}", flush=True)
    print(f"sum: per-z {tot['0']:.1f} us, zmap {tot['1']:.1f} us")


if __name__ == "__main__":
    main()
