"""Python call sites of the torch ops that still launch device work (fills, copies, adds, casts, cats) inside one
eager distill step (B = 2 x 10 s, the bench structure), recorded with a TorchFunctionMode: op name and the innermost
dphubert_amd frame, counted.  Every one of them becomes a graph node of the replayed step.

    python tools/aten_sites.py
"""
import collections
import sys
import traceback

import torch
from torch.overrides import TorchFunctionMode

sys.path.insert(0, ".")

WATCH = {"zeros", "zeros_like", "zero_", "fill_", "copy_", "clone", "cat", "stack", "add", "add_", "mul", "mul_",
         "to", "contiguous", "full", "ones", "ones_like", "sub", "div", "sum", "neg", "where", "index_select",
         "masked_fill", "masked_fill_", "narrow_copy", "float", "bfloat16", "new_zeros", "new_full", "__add__",
         "__mul__", "__sub__", "__truediv__", "__iadd__", "__imul__"}


class Rec(TorchFunctionMode):
    def __init__(self):
        super().__init__()
        self.sites = collections.Counter()

    def __torch_function__(self, func, types, args=(), kwargs=None):
        name = getattr(func, "__name__", str(func))
        if name in WATCH:
            dev = any(isinstance(a, torch.Tensor) and a.is_cuda for a in args) or \
                (kwargs or {}).get("device") is not None
            if dev:
                fr = [f for f in traceback.extract_stack()[:-1] if "dphubert_amd" in f.filename]
                where = f"{fr[-1].filename.split('/')[-1]}:{fr[-1].lineno} ({fr[-1].name})" if fr else "?"
                self.sites[(name, where)] += 1
        return func(*args, **(kwargs or {}))


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
    rec = Rec()
    with rec:
        tr.step(batch)
    torch.cuda.synchronize()
    tot = 0
    for (name, where), n in rec.sites.most_common():
        tot += n
        print(f"{n:4d}  {name:12s} {where}")
    print(f"total {tot} torch calls on CUDA tensors in one eager step")


if __name__ == "__main__":
    main()
