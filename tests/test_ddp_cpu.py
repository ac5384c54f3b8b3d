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
