"""Which Python call sites still launch ATen kernels (fill / zero / copy / add / cat) inside the distill step:
one eager HuBERT-Base step (B = 2 x 10 s: same structure as the bench step) under torch.profiler with stacks,
the ATen ops that launch device work grouped by their innermost dphubert_amd frames.

    python tools/aten_trace.py
"""
import sys
from collections import Counter

import torch

sys.path.insert(0, ".")

OPS = ("aten::fill_", "aten::zero_", "aten::copy_", "aten::add", "aten::add_", "aten::cat", "aten::mul",
       "aten::sum", "aten::div", "aten::clone", "aten::index", "aten::sub", "aten::neg", "aten::to")


def main():
    from dphubert_amd.synthetic import HUBERT_BASE_CONFIG, synthetic_batch
    from dphubert_amd.trainer import Trainer, build_distill_module
    dm = build_distill_module(HUBERT_BASE_CONFIG).cuda()
    dm.global_step = 5000
    tr = Trainer(dm, clip_norm=10.0)
    w, l = synthetic_batch(2, 160000)
    batch = (w.cuda(), l.cuda())
    for _ in range(2):
        tr.step(batch)
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], with_stack=True) as prof:
        tr.step(batch)
        torch.cuda.synchronize()
    sites = Counter()
    for ev in prof.events():
        if ev.name not in OPS:
            continue
        # only top-level ATen calls (not the ones nested in another ATen op)
        if ev.cpu_parent is not None and ev.cpu_parent.name.startswith("aten::"):
            continue
        fr = [s for s in (ev.stack or []) if "dphubert_amd" in s or "bench.py" in s]
        sites[(ev.name, " <- ".join(f.split("/")[-1] for f in fr[:3]))] += 1
    tot = 0
    for (name, where), n in sites.most_common():
        tot += n
        print(f"{n:4d}  {name:14s} {where}")
    print(f"total {tot} top-level ATen calls in one eager step")


if __name__ == "__main__":
    main()
