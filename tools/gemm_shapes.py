"""Per-shape GEMM time of one eager bench step (B=16 x 10 s): which shapes the step's GEMM time
goes to.  Run on the GPU box:  python tools/gemm_shapes.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from dphubert_amd import ops
    from dphubert_amd.kernels import LaunchProfiler
    from dphubert_amd.synthetic import HUBERT_BASE_CONFIG, synthetic_batch
    from dphubert_amd.trainer import Trainer, build_distill_module
    torch.cuda.set_device(0)
    ops.manual_seed(2022)
    m = build_distill_module(HUBERT_BASE_CONFIG, pruning_units="conv,head,interm", distill_layers="0.4,8,12",
                             use_reg=True)
    m.global_step = 5000
    m = m.cuda()
    tr = Trainer(m, clip_norm=10.0)
    w, l = synthetic_batch(16, 160000, seed=2022)
    batch = (w.cuda(), l.cuda())
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    prof = LaunchProfiler(by_shape=True)
    with prof:
        tr.step(batch)
    s = prof.summary()
    tot = sum(v["ms"] for v in s.values())
    print(f"total GEMM {tot:.3f} ms  ({sum(v['flops'] for v in s.values()) / tot / 1e9:.0f} TF/s)")
    for k, v in sorted(s.items(), key=lambda kv: -kv[1]["ms"]):
        print(f"{v['ms']:7.3f} ms {v['launches']:4d}x {v['ms'] / v['launches'] * 1e3:7.1f} us "
              f"{v['flops'] / v['ms'] / 1e9:6.0f} TF/s  {k}")


if __name__ == "__main__":
    main()
