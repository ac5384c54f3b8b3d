"""Bisect which part of the distill step breaks HIP-graph capture.

python tools/graph_bisect.py MODE   with MODE in
  gemm        one fused GEMM launch
  memset      dph_grad_sumsq (hipMemsetAsync node + kernel)
  teacher     teacher.extract_features (no grad)
  student     DistillModule.training_step (forward only)
  fwdbwd      training_step + backward
  full        + reducer.finish + optimizer.launch
Each mode: warm up eagerly, capture, replay twice, print OK.
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))


def capture(fn, name):
    torch.cuda.synchronize()
    from dphubert_amd import ops
    ops.reset_zero_arena()
    g = torch.cuda.CUDAGraph()
    print(f"[{name}] capture begin", flush=True)
    with torch.cuda.graph(g):
        out = fn()
    print(f"[{name}] capture end", flush=True)
    ops.reset_zero_arena()
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    print(f"[{name}] replay OK", flush=True)
    return out


def main(mode):
    torch.cuda.set_device(0)
    from dphubert_amd import kernels as K
    if mode == "gemm":
        x = torch.randn(512, 256, device="cuda").to(torch.bfloat16)
        w = torch.randn(384, 256, device="cuda").to(torch.bfloat16)
        K.linear_fwd(x, w)
        capture(lambda: K.linear_fwd(x, w, act=K.ACT_GELU), mode)
        return
    if mode == "memset":
        from dphubert_amd.optim import FusedAdamW
        ps = [torch.randn(1000, device="cuda", requires_grad=True)]
        opt = FusedAdamW(ps, lr=1e-3, max_grad_norm=1.0)
        ps[0].grad = torch.randn(1000, device="cuda")
        opt.step()
        capture(lambda: opt.launch(), mode)
        return
    from test_graph_gpu import _batch, _module
    from dphubert_amd.trainer import Trainer
    batch = _batch()
    dm = _module()
    tr = Trainer(dm, clip_norm=10.0)
    tr.step(batch)
    tr.step(batch)
    torch.cuda.synchronize()
    if mode == "teacher":
        def f():
            with torch.no_grad():
                return dm.teacher_model.extract_features(*batch)[0][-1]
        capture(f, mode)
    elif mode == "student":
        def f():
            with torch.no_grad():
                return dm.training_step(batch, 0)
        capture(f, mode)
    elif mode == "fwdbwd":
        def f():
            tr.reducer.prepare(zero=True, sync=True)
            loss = dm.training_step(batch, 0)
            loss.backward()
            return loss
        capture(f, mode)
    elif mode == "full":
        def f():
            return tr._gpu_step(batch, True)
        capture(f, mode)


if __name__ == "__main__":
    main(sys.argv[1])
