"""Data-parallel gradient path on CPU (gloo, world_size 2): GradReducer bucketing, fused-group
layout, direct gradient sinks (ops.GradOut) and gradient accumulation.

The RCCL path on the GPU is the same code with backend "nccl" (ReduceOp.AVG); here the reduction
is SUM + divide on gloo.  Reference: distill.py:41 (strategy="ddp"), SURVEY 8(e).
"""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dphubert_amd.ddp import GradReducer
from dphubert_amd.ops import GradOut


class SinkLinear(torch.autograd.Function):
    """y = x @ w^T + b whose weight/bias gradients go through GradOut (as the HIP Functions do)."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x)
        ctx.params = (w, b)
        return x @ w.t() + b

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        w, b = ctx.params
        go = GradOut(x.device)
        dw, direct = go.buf(w, zero=False)
        if direct:
            dw.add_(dy.t() @ x)
        else:
            dw.copy_(dy.t() @ x)
        db, _ = go.buf(b)
        db.add_(dy.sum(0))
        go.done()
        return dy @ w, go.ret(w), go.ret(b)


class DeferLinear(torch.autograd.Function):
    """SinkLinear whose weight gradient goes through ops._layer_wgrad: queued inside an ops.grouped_wgrads block
    (the encoder layers' path), its parameter held back from the reducer until the group lands."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x)
        ctx.params = (w, b)
        return x @ w.t() + b

    @staticmethod
    def backward(ctx, dy):
        from dphubert_amd import ops
        (x,) = ctx.saved_tensors
        w, b = ctx.params
        go = GradOut(x.device)
        dw, direct = go.buf(w, zero=False)
        if direct:
            assert ops._layer_wgrad(dy.contiguous(), x, dw, direct, (w,)) is None   # queued, not run
        else:
            dw.copy_(dy.t() @ x)
        db, _ = go.buf(b)
        db.add_(dy.sum(0))
        go.done()
        return dy @ w, go.ret(w), go.ret(b)


def _cpu_grouped(items, accumulate=True):
    """CPU stand-in for kernels.linear_wgrad_grouped (the HIP launch) in the gloo tests."""
    with torch.no_grad():     # (the HIP launch writes through pointers; the exit flush runs outside the backward)
        for dy, x, dw in items:
            if accumulate:
                dw.add_(dy.t() @ x)
            else:
                dw.copy_(dy.t() @ x)


class Net(torch.nn.Module):
    def __init__(self, sink: bool):
        super().__init__()
        g = torch.Generator().manual_seed(0)
        self.q = torch.nn.Linear(6, 4)
        self.k = torch.nn.Linear(6, 4)
        self.v = torch.nn.Linear(6, 4)
        self.o = torch.nn.Linear(12, 3)
        for p in self.parameters():
            with torch.no_grad():
                p.copy_(torch.randn(p.shape, generator=g))
        self.sink = sink

    def lin(self, m, x):
        if self.sink == "defer":
            return DeferLinear.apply(x, m.weight, m.bias)
        return SinkLinear.apply(x, m.weight, m.bias) if self.sink else m(x)

    def forward(self, x):
        h = torch.cat([self.lin(self.q, x), self.lin(self.k, x), self.lin(self.v, x)], dim=1)
        return (self.lin(self.o, torch.tanh(h)) ** 2).mean()

    def groups(self):
        return [(self.q.weight, self.k.weight, self.v.weight), (self.q.bias, self.k.bias, self.v.bias)]


def _inputs(rank, micro):
    g = torch.Generator().manual_seed(100 + 10 * rank + micro)
    return torch.randn(5, 6, generator=g)


def _reference_grads(world, accum):
    net = Net(sink=False)
    for r in range(world):
        for m in range(accum):
            (net(_inputs(r, m)) / accum).backward()
    return {n: p.grad / world for n, p in net.named_parameters()}


def _reference_abs_mean(world, accum):
    """mean over ranks of |rank's accumulated gradient| (the scale the bf16 rounding error is relative to)."""
    out = {}
    for r in range(world):
        net = Net(sink=False)
        for m in range(accum):
            (net(_inputs(r, m)) / accum).backward()
        for n, p in net.named_parameters():
            out[n] = out.get(n, 0) + p.grad.abs() / world
    return out


def _worker(rank, world, port, sink, accum, bucket_mb, q, comm="fp32"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        net = Net(sink=sink)
        red = GradReducer(list(net.parameters()), bucket_mb=bucket_mb, groups=net.groups(),
                          comm_dtype=torch.bfloat16 if comm == "bf16" else torch.float32)
        from dphubert_amd import ops
        if sink == "defer":
            ops.K.linear_wgrad_grouped = _cpu_grouped
        for m in range(accum):
            red.prepare(zero=m == 0, sync=m + 1 == accum)
            with ops.grouped_wgrads(2 if sink == "defer" else 1):
                (net(_inputs(rank, m)) / accum).backward()
            assert not any(getattr(p, "_dph_hold", False) for p in net.parameters())
        red.finish()
        # fused groups are laid out back-to-back in one bucket
        for grp in net.groups():
            ptrs = [p.grad.data_ptr() for p in grp]
            sizes = [p.numel() * 4 for p in grp]
            assert all(ptrs[i] + sizes[i] == ptrs[i + 1] for i in range(len(grp) - 1))
        q.put((rank, {n: p.grad.detach().numpy().copy() for n, p in net.named_parameters()}))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("sink,accum,bucket_mb,comm", [(False, 1, 64.0, "fp32"), (True, 1, 64.0, "fp32"),
                                                       (True, 2, 1e-4, "fp32"), (False, 3, 1e-4, "fp32"),
                                                       (True, 1, 64.0, "bf16"), (True, 3, 1e-4, "bf16"),
                                                       (False, 2, 64.0, "bf16"), ("defer", 1, 1e-4, "fp32"),
                                                       ("defer", 2, 64.0, "fp32")])
def test_grad_reducer_gloo_ws2(sink, accum, bucket_mb, comm):
    """fp32 payload: exact mean of the ranks' accumulated gradients ("defer": the weight gradients queued by
    ops.grouped_wgrads and launched two at a time, their buckets' collectives held until they land).  bf16 payload (half the link
    bytes): each rank's accumulated gradient is rounded to bf16 (8 mantissa bits) before the sum, so the mean
    is within 2 bf16 ulps (2 * 2^-8 relative) of the exact one, elementwise."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sink, accum, bucket_mb, q, comm))
             for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _reference_grads(world, accum)
    for r in range(world):
        for n, g in want.items():
            x = torch.from_numpy(got[r][n])
            if comm == "bf16":
                bound = 2 * 2.0 ** -8 * _reference_abs_mean(world, accum)[n] + 1e-6
                assert ((x - g).abs() <= bound).all(), (r, n, (x - g).abs().max())
                assert torch.equal(torch.from_numpy(got[0][n]), x)   # every rank holds the same reduced values
            else:
                assert torch.allclose(x, g, rtol=1e-5, atol=1e-6), (r, n)


def test_grad_out_fallback_without_reducer():
    """No reducer armed: GradOut hands out fresh tensors and autograd accumulates as usual."""
    net = Net(sink=True)
    ref = Net(sink=False)
    x = _inputs(0, 0)
    net(x).backward()
    ref(x).backward()
    for (n, p), (_, r) in zip(net.named_parameters(), ref.named_parameters()):
        assert torch.allclose(p.grad, r.grad, rtol=1e-5, atol=1e-6), n


def test_bucket_units_16_byte_aligned():
    """Every parameter unit starts on a 16-byte boundary of its bucket (the weight-gradient kernels store whole
    16-byte vectors into the bucket), also after odd-sized parameters (a scalar layer mask, a 3-wide bias); a
    fused group (q / k / v) stays back to back."""
    ps = [torch.nn.Parameter(torch.zeros(s)) for s in [(1,), (3,), (8, 4), (5,), (6, 2), (6, 2), (6, 2), (1,)]]
    red = GradReducer(ps, bucket_mb=1e-4, groups=[tuple(ps[4:7])])
    assert sum(f.numel() for f in red.flat) >= sum(p.numel() for p in ps)
    for p in ps:
        assert red.offsets[id(p)] % 4 == 0 or any(p is q for q in ps[5:7]), (p.shape, red.offsets[id(p)])
    o = [red.offsets[id(p)] for p in ps[4:7]]
    assert red.bucket_of[id(ps[4])] == red.bucket_of[id(ps[6])] and o[1] == o[0] + 12 and o[2] == o[1] + 12
    red.remove()


# ---------------------------------------------------------------------------------------------
# the comm window: encoder buckets' collectives before the frontend backward
# ---------------------------------------------------------------------------------------------
_EVENTS = []


class FrontLinear(SinkLinear):
    """The 'frontend' below the encoder: its backward start is recorded."""

    @staticmethod
    def backward(ctx, dy):
        _EVENTS.append(("frontend",))
        return SinkLinear.backward(ctx, dy)


class Stack(torch.nn.Module):
    """frontend -> ops.mark_encoder_input -> 12 'encoder layers' whose weight gradients are deferred (DeferLinear)."""

    def __init__(self, n_layers=12):
        super().__init__()
        g = torch.Generator().manual_seed(1)
        self.front = torch.nn.Linear(6, 8)
        self.layers = torch.nn.ModuleList([torch.nn.Linear(8, 8) for _ in range(n_layers)])
        for p in self.parameters():
            with torch.no_grad():
                p.copy_(torch.randn(p.shape, generator=g) * 0.5)

    def forward(self, x):
        from dphubert_amd import ops
        h = ops.mark_encoder_input(FrontLinear.apply(x, self.front.weight, self.front.bias))
        for lay in self.layers:
            h = torch.tanh(DeferLinear.apply(h, lay.weight, lay.bias))
        return (h ** 2).mean()


def _window_worker(rank, world, port, group, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dphubert_amd import ops
        ops.K.linear_wgrad_grouped = _cpu_grouped
        net = Stack()
        # one bucket per layer (8x8 + 8 floats = 288 B): each layer's collective is its own event
        red = GradReducer(list(net.parameters()), bucket_mb=300 / 2 ** 20)
        orig = red._launch

        def launch(bi):
            _EVENTS.append(("launch", bi))
            return orig(bi)

        red._launch = launch
        red.prepare()
        with ops.grouped_wgrads(group):
            net(_inputs(rank, 0)[:, :6]).backward()
        red.finish()
        enc = {red.bucket_of[id(lay.weight)] for lay in net.layers}
        q.put((rank, list(_EVENTS), sorted(enc)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("group", [6, 5])
def test_encoder_buckets_reduce_before_frontend_backward(group):
    """DPH_WGRAD_GROUP=6 (and 5, which does not divide the 12 layers): every encoder bucket's all-reduce is issued
    before the frontend backward starts -- the last partial group is flushed by the hook on the encoder input
    (ops.mark_encoder_input), not at the end of the backward -- so the collectives overlap the frontend backward."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_window_worker, args=(r, world, port, group, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ev, enc in res:
        front = ev.index(("frontend",))
        launched = {e[1] for e in ev[:front] if e[0] == "launch"}
        assert set(enc) <= launched, (rank, group, ev)


def _replica_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dphubert_amd.ddp import broadcast_module, verify_replicas
        torch.manual_seed(10 + rank)                   # every rank initialises differently
        net = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.BatchNorm1d(5), torch.nn.Linear(5, 3))
        net[1].running_mean.normal_()
        v0 = net[0].weight._version
        broadcast_module(net)
        assert net[0].weight._version > v0             # the bf16 image caches key on the version
        verify_replicas(net)                           # identical now: no error
        # numpy copies travel through the queue by value (torch tensors go by shared-memory handle, which a worker
        # that has exited no longer holds)
        state = {k: v.detach().numpy().copy() for k, v in net.state_dict().items()}
        if rank == 1:
            with torch.no_grad():
                net[2].weight[0, 0] += 1e-6            # one element on one rank
        try:
            verify_replicas(net)
            mismatch = None
        except RuntimeError as e:
            mismatch = str(e)
        q.put((rank, state, mismatch))
    finally:
        dist.destroy_process_group()


def test_broadcast_and_verify_replicas_gloo_ws2():
    """Trainer construction broadcasts rank 0's parameters and buffers (torch DDP's construction-time broadcast,
    distill.py:41); verify_replicas (run after a checkpoint load) fails on every rank when one element differs."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_replica_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (s, m)) for r, s, m in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k in res[0][0]:
        assert (res[0][0][k] == res[1][0][k]).all(), k
    for r in range(world):
        assert res[r][1] is not None and "2.weight" in res[r][1], res[r][1]


def test_wgrad_group_plan_and_bucket_order():
    """The bucket layout follows the predicted gradient-ready order (distill projections first; HardConcrete logits
    and Lagrange multipliers, whose gradients land at the end of the backward, in the last bucket), and the planned
    weight-gradient group minimises the modelled step end: the whole encoder at world size 1, no larger a group on a
    slow link than on a fast one."""
    from dphubert_amd.synthetic import HUBERT_BASE_CONFIG
    from dphubert_amd import trainer as T
    dm = T.build_distill_module(HUBERT_BASE_CONFIG, distill_layers="0.4,8,12")
    opt = dm.configure_optimizers(clip_norm=10.0)["optimizer"]
    params = [p for g in opt.param_groups for p in g["params"]]
    red = GradReducer(list(reversed(T.grad_ready_order(dm, params))), groups=T.fused_grad_groups(dm.student_model))
    names = {id(p): n for n, p in dm.named_parameters()}
    first, last = [names[id(p)] for p in red.buckets[0]], [names[id(p)] for p in red.buckets[-1]]
    assert any(n.startswith("distill_linear_projs") for n in first)
    assert all("log_alpha" in n or n.startswith("lambda") or "feature_extractor" in n or "encoder." in n for n in last)
    assert sum("log_alpha" in n for n in last) == sum("log_alpha" in n for n in names.values())
    proj = list(dm.distill_linear_projs.parameters())
    frames = 16 * 160000 / 320
    assert T.plan_wgrad_group(dm.student_model, red.buckets, 1, frames) == 12
    picks = {}
    for bus in (150.0, 20.0):
        g = T.plan_wgrad_group(dm.student_model, red.buckets, 8, frames, bus, 4, proj)
        ends = {c: max(T.wgrad_group_timeline(dm.student_model, red.buckets, 8, frames, c, bus, 4, proj))
                for c in (1, 2, 3, 4, 6, 8, 12)}
        assert ends[g] <= min(ends.values()) + 1e-9, (bus, g, ends)
        picks[bus] = g
    assert picks[20.0] <= picks[150.0], picks


def _plan_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.pop("DPH_XGMI_BUS_GBPS", None)
    os.environ.pop("DPH_WGRAD_GROUP", None)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dphubert_amd.synthetic import HUBERT_BASE_CONFIG
        from dphubert_amd import trainer as T
        dm = T.build_distill_module(HUBERT_BASE_CONFIG, distill_layers="0.4,8,12")
        tr = T.Trainer(dm, clip_norm=10.0)
        # the bucketed loader hands every rank its own padded length: 16 x 10 s here, 3 x 2 s there
        B, S = (16, 160000) if rank == 0 else (3, 32000)
        local = T.plan_wgrad_group(dm.student_model, tr.reducer.buckets, world, B * S / 320.0, T.XGMI_BUS_GBPS, 4,
                                   list(dm.distill_linear_projs.parameters()))
        tr._plan((torch.zeros(B, S), None))
        ready, _, t_end = T.grad_ready_times(dm.student_model, tr.wgrad_plan["frames"], tr.wgrad_group,
                                             list(dm.distill_linear_projs.parameters()))
        order = sorted(range(len(tr.reducer.buckets)),
                       key=lambda bi: (max(ready.get(id(p), t_end) for p in tr.reducer.buckets[bi]), bi))
        q.put((rank, local, tr.wgrad_group, tr.wgrad_plan["frames"], order))
    finally:
        dist.destroy_process_group()


def test_wgrad_group_plan_identical_across_ranks():
    """ranks with different padded lengths must plan the same weight-gradient group -- it
    decides when the held-back encoder gradients land and so the order of the bucket collectives.  The plan runs on
    the MAX frame count over the ranks: the group, the frames it was planned on and the predicted bucket launch
    order agree on both ranks, although each rank's own frames would have picked different groups."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_plan_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (loc, g, f, o)) for r, loc, g, f, o in (q.get(timeout=300) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][0] != res[1][0], f"precondition: local plans should differ ({res})"
    assert res[0][1] == res[1][1] == res[0][0], res       # rank 0 has the larger batch: its plan wins
    assert res[0][2] == res[1][2] == 16 * 160000 / 320.0
    assert res[0][3] == res[1][3]


def _capture_count_worker(rank, world, port, accum, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dphubert_amd import ops
        ops.K.linear_wgrad_grouped = _cpu_grouped
        net = Net(sink="defer")
        red = GradReducer(list(net.parameters()), bucket_mb=1e-4, groups=net.groups())
        calls = []
        orig = dist.all_reduce

        def counting(t, *a, **kw):
            calls.append(t.data_ptr())
            return orig(t, *a, **kw)

        dist.all_reduce = counting
        per_micro = []
        for step in range(2):                       # two optimizer steps
            for m in range(accum):
                zero, final = m == 0, m + 1 == accum
                n0 = len(calls)
                # the body Trainer._gpu_step records into the (zero, final) graph: prepare, backward inside
                # grouped_wgrads, and on the final micro-step finish() (what the captured graph replays)
                red.prepare(zero=zero, sync=final)
                with ops.grouped_wgrads(2):
                    (net(_inputs(rank, m)) / accum).backward()
                if final:
                    red.finish()
                per_micro.append((step, m, calls[n0:]))
        dist.all_reduce = orig
        flat = [f.data_ptr() for f in red.flat]
        q.put((rank, [(s, m, [flat.index(c) for c in cs]) for s, m, cs in per_micro], len(red.flat)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("accum", [1, 3])
def test_reducer_collectives_once_per_optimizer_step(accum):
    """The body of each captured micro-step graph (Trainer._gpu_step: reducer.prepare(zero, sync=final), the
    backward inside ops.grouped_wgrads, finish() on the final micro-step) issues every bucket's collective exactly
    once per optimizer step -- none on the non-final micro-steps of gradient accumulation (run_large.sh:54), each
    bucket once on the final one, in the same order on both ranks -- so the graph replay of that body does too."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_capture_count_worker, args=(r, world, port, accum, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (pm, nb)) for r, pm, nb in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        pm, nb = res[r]
        assert nb > 1
        for step, m, buckets in pm:
            if m + 1 < accum:
                assert buckets == [], (r, step, m, buckets)
            else:
                assert sorted(buckets) == list(range(nb)), (r, step, m, buckets)
    assert res[0][0] == res[1][0]
