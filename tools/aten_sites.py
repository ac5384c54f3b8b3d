"""Every ATen op that launches device work in one eager distill step (B = 2 x 10 s HuBERT-Base, the bench step's
structure), by op and innermost dphubert_amd call site -- logged by a TorchDispatchMode (factories such as
torch.zeros count as their fill), so the captured step graph's Fill / copyBuffer / elementwise nodes can be traced
to the Python line that adds them.

    python tools/aten_sites.py
"""
import sys
import traceback
from collections import Counter

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, ".")

DEVICE_OPS = ("fill", "zero", "copy", "add", "cat", "mul", "sum", "div", "clone", "index", "sub", "neg", "_to_copy",
              "zeros", "ones", "full", "where", "masked", "clamp", "stack", "mean", "sqrt", "pow", "lerp", "addcmul",
              "scatter", "gather", "narrow_copy", "cumsum", "max", "min", "abs", "exp", "log", "rsub", "new_zeros")


class Sites(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.sites = Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        out = func(*args, **kwargs)
        name = func.overloadpacket.__name__
        if any(k in name for k in DEVICE_OPS):
            dev = any(isinstance(a, torch.Tensor) and a.is_cuda for a in list(args) + list(kwargs.values()))
            dev = dev or (isinstance(out, torch.Tensor) and out.is_cuda)
            if dev:
                fr = [f for f in traceback.extract_stack() if "dphubert_amd" in f.filename or "torch/autograd" in
                      f.filename]
                where = " <- ".join(f"{f.filename.split('/')[-1]}:{f.lineno}" for f in reversed(fr[-3:]))
                self.sites[(name, where)] += 1
        return out


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
    mode = Sites()
    with mode:
        tr.step(batch)
    torch.cuda.synchronize()
    tot = 0
    for (name, where), n in mode.sites.most_common():
        tot += n
        print(f"{n:4d}  {name:16s} {where}")
    print(f"total {tot} device ATen ops in one eager step")


if __name__ == "__main__":
    main()
