"""Which Python call sites launch the small ATen kernels of an eager bench step (fills, adds,
copies, int64 length math).  Run on the GPU box:  python tools/torch_ops.py"""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from dphubert_amd import ops
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
    import collections
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    cnt = collections.Counter()

    class Log(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            name = str(func.overloadpacket)
            kern = ("fill", "zero", "add", "copy", "sub", "div", "mul", "cat", "clamp", "remainder", "floor",
                    "where", "lt", "ge", "gt", "le", "sum", "index", "arange", "_to_copy", "ones", "full", "neg", "rsub")
            if any(k in name for k in kern):
                fr = [f for f in traceback.extract_stack()[:-1] if "dphubert_amd" in f.filename]
                where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in fr[-3:][::-1])
                cnt[(name, where)] += 1
            return func(*args, **(kwargs or {}))

    with Log():
        tr.step(batch)
        torch.cuda.synchronize()
    for (name, where), c in cnt.most_common(40):
        print(f"{c:4d}  {name:28s} {where}")
    # backward-thread ops: attribute to the enclosing autograd node via the profiler's CPU parents
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        tr.step(batch)
        torch.cuda.synchronize()
    c2 = collections.Counter()
    for ev in prof.events():
        if ev.name in ("aten::fill_", "aten::zero_", "aten::add", "aten::add_", "aten::copy_", "aten::mul",
                       "aten::sub", "aten::div", "aten::cat"):
            chain, par = [], ev.cpu_parent
            while par is not None and len(chain) < 6:
                chain.append(par.name)
                par = par.cpu_parent
            top = [c for c in chain if "Backward" in c or "evaluate_function" in c or "AccumulateGrad" in c]
            if ev.cpu_parent is not None and ev.cpu_parent.name.startswith("aten::"):
                continue   # nested inside another aten op (counted there)
            c2[(ev.name, " <- ".join(chain[:3]))] += 1
    print("--- by parent ---")
    for (name, where), c in c2.most_common(40):
        print(f"{c:4d}  {name:16s} {where}")

if __name__ == "__main__":
    main()
