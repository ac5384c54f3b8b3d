"""Data-parallel gradient reduction over RCCL (xGMI), overlapped with backward.

Replaces PyTorch-Lightning ``strategy="ddp"`` (distill.py:41 -> torch DDP over
NCCL).  Design for one 8x MI355X node:

* gradients of the trainable parameters (student + HardConcrete log_alpha +
  distill projections + Lagrange multipliers, ~95.6 M fp32 = 382 MB for
  HuBERT-Base) live in a few large flat buckets; each ``p.grad`` is a view
  into its bucket, so the all-reduce needs no pack/unpack copies;
* buckets are filled in reverse registration order (= backward order), and a
  bucket's ``all_reduce`` is launched asynchronously from the
  post-accumulate-grad hook of its last parameter, so RCCL traffic over the
  point-to-point xGMI links overlaps the remaining backward kernels;
* bucket size defaults to 64 MB: the ring all-reduce on xGMI is per-link
  bound, so few large collectives beat DDP's 25 MB default;
* the average is applied in the collective (``ReduceOp.AVG``) on RCCL, or by
  a scale after SUM on gloo (CPU tests);
* ``comm_dtype=torch.bfloat16`` halves the payload on the links (191 MB
  instead of 382 MB per step): each bucket is cast to a persistent bf16 buffer right
  before its collective and cast back into the fp32 bucket after it; the optimizer
  still reads fp32 gradients (masters and moments stay fp32);
* replicas start identical: ``broadcast_module`` sends rank 0's parameters and buffers at
  trainer construction (DDP's construction-time broadcast), ``verify_replicas`` checks them
  after a checkpoint load.
"""

from typing import Iterable, List, Optional, Sequence

import torch
import torch.distributed as dist


class GradReducer:
    """Flat-bucket gradient all-reduce, launched from gradient-ready notifications.

    ``groups``: tuples of parameters whose gradients must be laid out back-to-back, in the given
    order (e.g. q/k/v projection weights, produced by one fused weight-gradient GEMM).
    ``direct``: arm gradient sinks (``p._dph_sink``) so the HIP backward kernels accumulate
    straight into the bucket storage (ops.GradOut); autograd then never zero-fills or adds those
    gradients, and the Function notifies readiness through ``p._dph_sink_ready``.
    """

    def __init__(self, params: Iterable[torch.nn.Parameter], bucket_mb: float = 64.0, process_group=None,
                 groups: Optional[Sequence[Sequence[torch.nn.Parameter]]] = None, direct: bool = True,
                 comm_dtype: torch.dtype = torch.float32):
        if comm_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"comm_dtype must be float32 or bfloat16, got {comm_dtype}")
        self.comm_dtype = comm_dtype
        self.group = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        ps: List[torch.nn.Parameter] = []
        seen = set()
        for p in params:
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                ps.append(p)
        ps = list(reversed(ps))        # backward produces gradients roughly in reverse order
        group_of = {}
        for gi, grp in enumerate(groups or []):
            if all(id(p) in seen for p in grp):
                for p in grp:
                    group_of[id(p)] = gi
        units: List[List[torch.nn.Parameter]] = []
        placed = set()
        for p in ps:
            if id(p) in placed:
                continue
            unit = list(groups[group_of[id(p)]]) if id(p) in group_of else [p]
            placed.update(id(q) for q in unit)
            units.append(unit)
        self.params = [p for u in units for p in u]
        cap = int(bucket_mb * 1024 * 1024 / 4)
        self.buckets: List[List[torch.nn.Parameter]] = []
        # each unit starts on a 16-byte boundary of its bucket (the weight-gradient kernels store whole 16-byte
        # vectors straight into the bucket; a scalar layer-mask parameter would otherwise shift every later view)
        pad = lambda n: (n + 3) & ~3  # noqa: E731
        offsets = {}
        cur, n = [], 0
        for u in units:
            un = sum(p.numel() for p in u)
            if cur and n + un > cap:
                self.buckets.append(cur)
                cur, n = [], 0
            for p in u:
                offsets[id(p)] = n
                n += p.numel()
            n = pad(n)
            cur.extend(u)
        if cur:
            self.buckets.append(cur)
        self.flat = []
        self.bucket_of = {}
        for bi, b in enumerate(self.buckets):
            dev = b[0].device
            dt = b[0].dtype
            size = pad(max(offsets[id(p)] + p.numel() for p in b))
            self.flat.append(torch.zeros(size, dtype=dt, device=dev))
            for p in b:
                self.bucket_of[id(p)] = bi
        self.views = {}
        self.offsets = {}
        for bi, b in enumerate(self.buckets):
            for p in b:
                off = offsets[id(p)]
                self.views[id(p)] = self.flat[bi][off:off + p.numel()].view_as(p)
                self.offsets[id(p)] = off
        self.direct = direct
        self._pending = [0] * len(self.buckets)
        self._handles = [None] * len(self.buckets)
        self._hooks = [p.register_post_accumulate_grad_hook(self._hook) for p in self.params]
        self.backend = dist.get_backend(process_group) if dist.is_initialized() else None
        self.enabled = self.world > 1
        # persistent bf16 payload buffers (allocated once: a captured HIP graph replays them by address)
        self.payload = [torch.empty(f.numel(), dtype=torch.bfloat16, device=f.device) if
                        (self.enabled and comm_dtype == torch.bfloat16) else None for f in self.flat]
        self.sync = True
        self._seen = set()

    def force_enable(self):
        """Run the collectives even at world size 1 (tests / probes of the RCCL path on one GPU)."""
        self.enabled = True
        self.payload = [torch.empty(f.numel(), dtype=torch.bfloat16, device=f.device) if
                        self.comm_dtype == torch.bfloat16 else None for f in self.flat]

    def prepare(self, zero: bool = True, sync: bool = True):
        """Point every .grad at its bucket view (zeroed when ``zero``) before a backward.

        ``sync=False`` for the non-final micro-batches of gradient accumulation: gradients
        accumulate locally and no collective is launched until the final micro-batch.
        """
        if zero:
            self._zero_buckets()
        # buckets hold only this micro-batch's gradients (kernels may read a fresh weight gradient back: ops)
        self.fresh = bool(zero)
        for p in self.params:
            p.grad = self.views[id(p)]
            if self.direct:
                p._dph_sink = (self.flat[self.bucket_of[id(p)]], self.offsets[id(p)], tuple(p.shape))
                p._dph_sink_ready = self._ready
        self.sync = sync
        self._seen = set()
        self._pending = [len(b) for b in self.buckets]
        self._handles = [None] * len(self.buckets)

    def _zero_buckets(self):
        """All fp32 CUDA buckets zeroed by ONE dph_copy_f32_multi launch (instead of an ATen fill per
        bucket); CPU buckets (gloo tests) by torch."""
        cuda = [f for f in self.flat if f.is_cuda and f.dtype == torch.float32]
        for f in self.flat:
            if not (f.is_cuda and f.dtype == torch.float32):
                f.zero_()
        if not cuda:
            return
        if getattr(self, "_zero_tab", None) is None:
            from . import ops
            self._zero_rows = [(0, f.data_ptr(), f.numel()) for f in cuda]
            self._zero_tab = ops._table(self._zero_rows)
        from ._lib import call, ptr, stream_ptr
        call("dph_copy_f32_multi", ptr(self._zero_tab), len(self._zero_rows), max(r[2] for r in self._zero_rows),
             stream_ptr())

    def _hook(self, p):
        # also fires (with the bucket view untouched) for a parameter whose Function returned None
        # after writing through its sink; _ready() counts each parameter once per backward
        if p.grad is not self.views[id(p)] and p.grad.data_ptr() != self.views[id(p)].data_ptr():
            # autograd replaced the grad tensor (e.g. prepare() not called): copy into the bucket
            self.views[id(p)].copy_(p.grad)
            p.grad = self.views[id(p)]
        self._ready(p)

    def _ready(self, p):
        # (_dph_hold: the parameter's gradient GEMM is queued in an ops.grouped_wgrads block, which notifies again
        # once it has landed)
        # (_dph_defer_hold: its bias / LayerNorm-affine column reduction is queued in an ops.deferred_reductions block,
        # which notifies once the flush has written it)
        if not self.sync or id(p) in self._seen or getattr(p, "_dph_hold", False) or \
                getattr(p, "_dph_defer_hold", False):
            return
        self._seen.add(id(p))
        bi = self.bucket_of[id(p)]
        self._pending[bi] -= 1
        if self._pending[bi] == 0 and self.enabled:
            self._launch(bi)

    def _launch(self, bi):
        # a bucket may hold gradients written on the weight-gradient side stream (ops.wgrad_side): its collective
        # starts after them too
        from .ops import _WGRAD_SIDE
        side = _WGRAD_SIDE[0]
        if side is not None and side != torch.cuda.current_stream():
            torch.cuda.current_stream().wait_stream(side)
        f = self.flat[bi]
        if self.payload[bi] is not None:
            f = self.payload[bi]
            f.copy_(self.flat[bi])                 # stream-ordered after the bucket's last gradient kernel
        if self.backend == "nccl":
            self._handles[bi] = dist.all_reduce(f, op=dist.ReduceOp.AVG, group=self.group, async_op=True)
        else:
            self._handles[bi] = dist.all_reduce(f, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def finish(self):
        """Wait for every bucket (launch the ones whose params got no gradient) and average."""
        if not self.enabled:
            return
        for bi in range(len(self.buckets)):
            if self._handles[bi] is None:
                self._launch(bi)
        for bi, h in enumerate(self._handles):
            h.wait()
            if self.payload[bi] is not None:
                self.flat[bi].copy_(self.payload[bi])
            if self.backend != "nccl":
                self.flat[bi].div_(self.world)
        for p in self.params:
            p.grad = self.views[id(p)]

    def remove(self):
        for h in self._hooks:
            h.remove()
        for p in self.params:
            for a in ("_dph_sink", "_dph_sink_ready"):
                if hasattr(p, a):
                    delattr(p, a)


# ---------------------------------------------------------------------------------------------
# replica consistency (torch DDP's construction-time broadcast, distill.py:41 strategy="ddp")
# ---------------------------------------------------------------------------------------------
def _module_tensors(module: torch.nn.Module):
    """(name, tensor) of every parameter and buffer, each storage once."""
    seen, out = set(), []
    for n, t in list(module.named_parameters()) + list(module.named_buffers()):
        if t is None or t.data_ptr() in seen or t.numel() == 0:
            continue
        seen.add(t.data_ptr())
        out.append((n, t))
    return out


def broadcast_module(module: torch.nn.Module, src: int = 0, process_group=None):
    """Every parameter and buffer of ``module`` from rank ``src``: flattened per (device, dtype) into one buffer and
    broadcast once each (a few large collectives, not one per tensor), then copied back in place under no_grad so
    each parameter's version moves (the cached bf16 GEMM images, keyed by version, are rebuilt)."""
    if not dist.is_initialized() or dist.get_world_size(process_group) == 1:
        return
    from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors
    by = {}
    for _, t in _module_tensors(module):
        by.setdefault((t.device, t.dtype), []).append(t)
    with torch.no_grad():
        for ts in by.values():
            flat = _flatten_dense_tensors([t.detach() for t in ts])
            dist.broadcast(flat, src, group=process_group)
            for t, v in zip(ts, _unflatten_dense_tensors(flat, ts)):
                t.copy_(v)


def replica_checksums(module: torch.nn.Module) -> torch.Tensor:
    """[2 * n_tensors] fp64: per tensor its sum and a position-weighted sum (weights 1..97 cycling, so a permutation
    or a shifted copy changes it)."""
    vals = []
    for _, t in _module_tensors(module):
        x = t.detach().reshape(-1).double()
        w = torch.arange(x.numel(), device=x.device, dtype=torch.float64).remainder_(97).add_(1.0)
        vals.append(torch.stack([x.sum(), (x * w).sum()]))
    return torch.cat(vals) if vals else torch.zeros(0, dtype=torch.float64)


def verify_replicas(module: torch.nn.Module, process_group=None, rtol: float = 0.0):
    """Raise on every rank if any parameter / buffer differs between ranks (checksums all-reduced MAX and MIN): after
    a checkpoint load (cli --resume_checkpoint) every rank must hold rank 0's state."""
    if not dist.is_initialized() or dist.get_world_size(process_group) == 1:
        return
    cs = replica_checksums(module)
    hi, lo = cs.clone(), cs.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=process_group)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=process_group)
    bad = ((hi - lo).abs() > rtol * hi.abs()).reshape(-1, 2).any(1).nonzero().flatten().tolist()
    if bad:
        names = [n for n, _ in _module_tensors(module)]
        raise RuntimeError(f"replicas differ across ranks in {len(bad)} tensors: {[names[i] for i in bad[:8]]}")
