"""The aten fills / copies left in one eager distill step (B = 2 x 10 s, the bench structure), by their innermost
dphubert_amd (or torch.autograd) frame: torch.profiler with stacks, ops aten::fill_ / zero_ / copy_ / clone /
_to_copy and their launches.  Catches the C++-side ones a TorchFunctionMode does not see (AccumulateGrad copies,
autograd zero-fills of undefined gradients, factory zeros inside Functions).

    python tools/fill_sites.py
"""
import collections
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, ".")

OPS = {"aten::fill_", "aten::zero_", "aten::copy_", "aten::clone", "aten::_to_copy", "aten::zeros", "aten::zeros_like",
       "aten::add_", "aten::cat"}


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
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        tr.step(batch)
        torch.cuda.synchronize()
    sites = collections.Counter()
    for ev in prof.events():
        if ev.name not in OPS or ev.device_type != torch.autograd.DeviceType.CPU:
            continue
        # the aten call that launched the device work itself (zeros -> zero_ -> fill_: counted at fill_)
        if not ev.kernels:
            continue
        st = [s for s in (ev.stack or []) if "dphubert_amd" in s or "autograd" in s]
        where = st[0].split("/")[-1] if st else "(no python frame: autograd engine)"
        # parent chain for the engine-side ones
        par, chain = ev.cpu_parent, []
        while par is not None and len(chain) < 3:
            chain.append(par.name)
            par = par.cpu_parent
        if not st:
            where += " <- " + " <- ".join(chain)
        sites[(ev.name, where)] += 1
    tot = 0
    for (name, where), n in sites.most_common():
        tot += n
        print(f"{n:4d}  {name:16s} {where}")
    print(f"total {tot}")
    kern = collections.Counter()
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA and ("Fill" in ev.name or "opy" in ev.name):
            kern[ev.name[:90]] += 1
    for k, n in kern.most_common(12):
        print(f"{n:4d}  kernel {k}")


if __name__ == "__main__":
    main()
