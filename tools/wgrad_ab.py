"""A/B of the weight-gradient GEMMs: the ping-pong (mn, mn) kernel with its tile / split plan (default) against
the register-staged kernel (DPH_GEMM_PPW=0), interleaved rounds in one process, outputs checked against each
other.  Shapes of the HuBERT-Base step at B = 16 x 10 s (T = 499 frames per utterance).

    python tools/wgrad_ab.py
"""
import os
import sys

import torch

sys.path.insert(0, ".")
from dphubert_amd import kernels as K  # noqa: E402

B, T = 16, 499
M = B * T
# (name, N_out, K_in, frames, conv (Lin, k, s) or None)
SHAPES = [
    ("qkv wgrad", 2304, 768, M, None),
    ("oproj wgrad", 768, 768, M, None),
    ("ffn1 wgrad", 3072, 768, M, None),
    ("ffn2 wgrad", 768, 3072, M, None),
    ("fproj wgrad", 768, 512, M, None),
    ("conv1 wgrad", 512, 3 * 512, B * 15999, (31999, 3, 2)),
    ("conv2 wgrad", 512, 3 * 512, B * 7999, (15999, 3, 2)),
    ("conv3 wgrad", 512, 3 * 512, B * 3999, (7999, 3, 2)),
    ("conv4 wgrad", 512, 3 * 512, B * 1999, (3999, 3, 2)),
    ("conv5 wgrad", 512, 2 * 512, B * 999, (1999, 2, 2)),
    ("conv6 wgrad", 512, 2 * 512, B * 499, (999, 2, 2)),
]


def main():
    rounds, iters = 3, 10
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    tot = {"ppw": 0.0, "old": 0.0}
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
        outs = {p: torch.zeros(n, kin, device="cuda") for p in tot}
        times = {p: [] for p in tot}
        info = {}

        def f(p, out):
            if p == "old":
                os.environ["DPH_GEMM_PPW"] = "0"
            else:
                os.environ.pop("DPH_GEMM_PPW", None)
            splits = K.choose_splits(n, kin, frames)
            info[p] = splits
            return K.gemm(K.dense(dy), Bm, K.dense(out), n, kin, frames, a_kcontig=False, b_kcontig=False,
                          c_dtype=K.OUT_F32, splits=splits)
        for p in tot:
            f(p, outs[p])
        torch.cuda.synchronize()
        for _ in range(rounds):
            for p in tot:
                keep = []
                e0.record()
                for _ in range(iters):
                    keep.append(f(p, outs[p]))
                e1.record()
                torch.cuda.synchronize()
                times[p].append(e0.elapsed_time(e1) / iters)
        os.environ.pop("DPH_GEMM_PPW", None)
        ref = outs["old"]
        err = ((outs["ppw"] - ref).norm() / ref.norm()).item()
        row = f"{name:12s} {n:5d}x{kin:5d}x{frames:7d} "
        for p in tot:
            ms = min(times[p])
            tot[p] += ms
            row += f"| {p} s={info[p]:2d} {ms * 1e3:7.1f} us {2 * n * kin * frames / ms / 1e9:5.0f} TF "
        print(row + f"| e={err:.1e}", flush=True)
        assert err < 1e-4, (name, err)
    print(f"sum: ppw {tot['ppw'] * 1e3:.1f} us, old {tot['old'] * 1e3:.1f} us")


if __name__ == "__main__":
    main()
