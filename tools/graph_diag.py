"""Diagnostics: where does a replayed step graph depart from an eager step?

Part ``rccl`` (2-layer module of tests/test_graph_gpu.py, world size 1 over RCCL): two eager trainers and one
graph trainer in lockstep; after every step, per-parameter gradient (bucket) / parameter / AdamW-moment
differences graph-vs-eager next to eager-vs-eager, and the clip norm of each trainer.

Part ``prof`` (bench shape): the main step graph and the profiled (event-node) graph replayed alternately, the
logged loss terms of each replay printed.

    python tools/graph_diag.py --part rccl [--no-force] [--chaotic]
    python tools/graph_diag.py --part prof [--batch 16]
"""
import argparse
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def rel(x, y):
    x, y = x.detach().double(), y.detach().double()
    return ((x - y).norm() / y.norm().clamp_min(1e-30)).item()


def snapshot(tr):
    m = tr.module
    out = {}
    for n, p in m.named_parameters():
        if not p.requires_grad:
            continue
        st = tr.optimizer.state.get(p, {})
        out[n] = (p.detach().clone(), tr.reducer.views[id(p)].detach().clone(),
                  st["exp_avg"].clone() if "exp_avg" in st else None)
    norm = tr.optimizer._sumsq[0].sqrt().item() if getattr(tr.optimizer, "_sumsq", None) is not None else None
    return out, norm


def compare(tag, se, se2, sg):
    (a, na), (b, nb), (g, ng) = se, se2, sg
    print(f"== {tag}: clip norm eager {na} eager2 {nb} graph {ng}")
    rows = []
    for k in a:
        for idx, what in ((0, "param"), (1, "grad"), (2, "exp_avg")):
            if a[k][idx] is None:
                continue
            e = rel(g[k][idx], a[k][idx])
            base = rel(b[k][idx], a[k][idx])
            rows.append((what, k, e, base))
    for what in ("grad", "param", "exp_avg"):
        rs = [r for r in rows if r[0] == what]
        cat = lambda d, i: torch.cat([d[k][i].double().flatten() for k in a if d[k][i] is not None])  # noqa: E731
        i = {"param": 0, "grad": 1, "exp_avg": 2}[what]
        print(f"   {what}: whole vector graph-vs-eager {rel(cat(g, i), cat(a, i)):.3e}  eager-vs-eager "
              f"{rel(cat(b, i), cat(a, i)):.3e}")
        rs.sort(key=lambda r: -(r[2] / max(r[3], 1e-12)))
        for r in rs[:8]:
            print(f"     {r[1]:70s} g-e {r[2]:.3e}  e-e {r[3]:.3e}")


def _ptr_values(obj, depth=0):
    """Every integer reachable from a ctypes argument (pointers inside structs, arrays, byref)."""
    import ctypes as C
    if depth > 4 or obj is None:
        return
    if isinstance(obj, bool):
        return
    if isinstance(obj, int):
        yield obj
    elif isinstance(obj, C._Pointer) or type(obj).__name__ == "CArgObject":
        inner = getattr(obj, "_obj", None)
        if inner is not None:
            yield from _ptr_values(inner, depth + 1)
    elif isinstance(obj, C.Structure):
        for f in obj._fields_:
            yield from _ptr_values(getattr(obj, f[0]), depth + 1)
    elif isinstance(obj, C.Array):
        for v in obj:
            yield from _ptr_values(v, depth + 1)
    elif isinstance(obj, (C.c_void_p, C.c_int64, C.c_uint64)):
        yield from _ptr_values(obj.value, depth + 1)


def watch_buckets():
    """Report every C-ABI call that passes a pointer into a gradient bucket whose all-reduce is already in
    flight (launched by GradReducer._launch, not yet joined by finish()): a kernel racing the collective."""
    import dphubert_amd._lib as L
    from dphubert_amd import ddp, kernels, ops, optim
    live = {}
    hits = []
    orig_call = L.call

    def call(name, *a):
        for v in _ptr_values(list(a)):
            for (rid, bi), (lo, hi) in list(live.items()):
                if lo <= v < hi:
                    hits.append((name, bi))
        return orig_call(name, *a)

    for m in (L, ops, kernels, optim):
        m.call = call
    orig_launch, orig_finish = ddp.GradReducer._launch, ddp.GradReducer.finish

    def _launch(self, bi):
        f = self.flat[bi]
        live[(id(self), bi)] = (f.data_ptr(), f.data_ptr() + f.numel() * f.element_size())
        return orig_launch(self, bi)

    def finish(self):
        r = orig_finish(self)
        for k in [k for k in live if k[0] == id(self)]:
            del live[k]
        return r

    ddp.GradReducer._launch = _launch
    ddp.GradReducer.finish = finish
    return hits


def part_rccl(args):
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(args.port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    hits = watch_buckets() if args.watch else None
    from test_graph_gpu import _batch, _module
    from dphubert_amd.trainer import Trainer
    batch = _batch()
    trs = [Trainer(_module(student_offset=not args.chaotic), clip_norm=10.0, graphs=(i == 2), graph_warmup=1)
           for i in range(3)]
    if args.force:
        for t in trs:
            t.reducer.force_enable()
    for step in range(args.steps):
        losses = [t.step(batch).item() for t in trs]
        torch.cuda.synchronize()
        print(f"step {step}: losses eager {losses[0]:.9f} eager2 {losses[1]:.9f} graph {losses[2]:.9f}")
        compare(f"after step {step}", snapshot(trs[0]), snapshot(trs[1]), snapshot(trs[2]))
        if hits is not None:
            from collections import Counter
            print(f"   calls touching an in-flight bucket so far: {dict(Counter(hits))}", flush=True)
    dist.destroy_process_group()


def part_prof(args):
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    from dphubert_amd import ops
    from dphubert_amd.kernels import LaunchProfiler
    from dphubert_amd.synthetic import HUBERT_BASE_CONFIG, synthetic_batch
    from dphubert_amd.trainer import Trainer, build_distill_module
    ops.manual_seed(2022)
    module = build_distill_module(HUBERT_BASE_CONFIG, pruning_units="conv,head,interm", distill_layers="0.4,8,12",
                                  use_reg=True)
    module.global_step = 5000
    module = module.to(dev)
    tr = Trainer(module, clip_norm=10.0, graphs=True, graph_warmup=2)
    wave, lengths = synthetic_batch(args.batch, int(args.seconds * 16000), seed=2022)
    batch = (wave.to(dev), lengths.to(dev))

    def show(tag, loss):
        torch.cuda.synchronize()
        terms = {k: round(float(v.float().sum()), 6) if torch.is_tensor(v) else v for k, v in module.logged.items()}
        print(f"{tag}: loss {loss.item():.6f} {terms}", flush=True)

    for i in range(3):
        show(f"warm {i}", tr.step(batch))
    if args.prof_graph:
        prof = LaunchProfiler()
        tr.prepare_profiled_step(prof)
    seq = args.seq.split(",")
    for i, s in enumerate(seq):
        show(f"{i} {s}", tr.step(batch, profiled=(s == "prof")))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--part", choices=["rccl", "prof"], default="rccl")
    ap.add_argument("--no-force", dest="force", action="store_false")
    ap.add_argument("--watch", action="store_true", help="report C-ABI calls that touch an in-flight bucket")
    ap.add_argument("--chaotic", action="store_true", help="student == teacher (the L1 sign chaos of run.sh's init)")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--port", type=int, default=29541)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--seq", default="main,main,prof,main,prof,prof")
    ap.add_argument("--no-prof-graph", dest="prof_graph", action="store_false")
    args = ap.parse_args()
    if args.part == "rccl":
        part_rccl(args)
    else:
        part_prof(args)


if __name__ == "__main__":
    main()
