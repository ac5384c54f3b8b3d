"""Fused AdamW + global-norm clipping on the GPU (torch.optim.AdamW semantics).

Drop-in for the optimizer built in lightning.py:200-228 (three param groups:
main / log_alpha / lambda with negative lr) plus Lightning's
``gradient_clip_val`` (distill.py:48).  One ``dph_grad_sumsq`` + one
``dph_adamw_step`` launch update every parameter; the clip coefficient never
leaves the device.
"""

import math
from typing import Iterable, List, Optional

import torch

from . import _lib
from ._lib import DphAdamGroup, DphTensorSlot, call, ptr

CHUNK = 8192   # must match optim.hip


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2,
                 max_grad_norm: Optional[float] = None):
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        if len(self.param_groups) > 4:
            raise ValueError("FusedAdamW supports at most 4 param groups")
        self.max_grad_norm = max_grad_norm
        self._chunk_key = None
        self._pinned = None
        self._slots_dev = None
        self._event = None
        self._step = 0

    def _params(self):
        out = []
        for gi, g in enumerate(self.param_groups):
            for p in g["params"]:
                out.append((gi, p))
        return out

    def _ensure_chunks(self, plist):
        key = tuple((p.data_ptr(), p.numel()) for _, p in plist)
        if key == self._chunk_key:
            return
        dev = plist[0][1].device
        cslot, cstart = [], []
        for si, (_, p) in enumerate(plist):
            n = p.numel()
            for s in range(0, n, CHUNK):
                cslot.append(si)
                cstart.append(s)
        self._cslot = torch.tensor(cslot, dtype=torch.int64, device=dev)
        self._cstart = torch.tensor(cstart, dtype=torch.int64, device=dev)
        self._nchunks = len(cslot)
        nbytes = len(plist) * C_SIZEOF_SLOT
        self._pinned = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        self._slots_dev = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        self._sumsq = torch.zeros(1, dtype=torch.float32, device=dev)
        self._chunk_key = key

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        plist = self._params()
        if not plist:
            return loss
        self._ensure_chunks(plist)
        # per-param state and the slot table (grad pointers change every step)
        if self._event is not None:
            self._event.synchronize()     # previous H2D copy of the pinned table is done
        slots = (DphTensorSlot * len(plist)).from_address(self._pinned.data_ptr())
        for i, (gi, p) in enumerate(plist):
            st = self.state[p]
            if len(st) == 0:
                st["step"] = torch.zeros((), dtype=torch.float32)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            if p.grad is not None and not p.grad.is_contiguous():
                p.grad = p.grad.contiguous()
            if p.grad is not None and p.grad.dtype != torch.float32:
                raise TypeError("FusedAdamW expects fp32 gradients")
            slots[i].param = p.data_ptr()
            slots[i].grad = p.grad.data_ptr() if p.grad is not None else 0
            slots[i].exp_avg = st["exp_avg"].data_ptr()
            slots[i].exp_avg_sq = st["exp_avg_sq"].data_ptr()
            slots[i].n = p.numel()
            slots[i].group = gi
            st["step"] += 1
        self._slots_dev.copy_(self._pinned, non_blocking=True)
        self._event = torch.cuda.Event()
        self._event.record()
        self._step += 1
        groups = (DphAdamGroup * 4)()
        for gi, g in enumerate(self.param_groups):
            groups[gi].lr = g["lr"]
            groups[gi].weight_decay = g["weight_decay"]
            groups[gi].beta1 = g["betas"][0]
            groups[gi].beta2 = g["betas"][1]
            groups[gi].eps = g["eps"]
        s = _lib.stream_ptr()
        clip = self.max_grad_norm is not None and self.max_grad_norm > 0
        if clip:
            call("dph_grad_sumsq", ptr(self._slots_dev), len(plist), ptr(self._cslot), ptr(self._cstart),
                 self._nchunks, ptr(self._sumsq), s)
        call("dph_adamw_step", ptr(self._slots_dev), len(plist), ptr(self._cslot), ptr(self._cstart), self._nchunks,
             groups, len(self.param_groups), self._step, ptr(self._sumsq) if clip else None,
             float(self.max_grad_norm or 0.0), s)
        return loss


import ctypes as _C  # noqa: E402

C_SIZEOF_SLOT = _C.sizeof(DphTensorSlot)


class LinearDecayLRScheduler(torch.optim.lr_scheduler.LRScheduler):
    """Linear warmup then linear decay (formula of lightning.py:37-44; the reference class itself
    passes a `verbose` kwarg that torch 2.10 removed)."""

    def __init__(self, optimizer, warmup_updates: int, max_updates: int, last_epoch: int = -1):
        self.warmup_updates = warmup_updates
        self.max_updates = max_updates
        super().__init__(optimizer, last_epoch=last_epoch)

    def get_lr(self):
        if self._step_count <= self.warmup_updates:
            return [self._step_count / self.warmup_updates * base_lr for base_lr in self.base_lrs]
        elif self._step_count >= self.max_updates:
            return [0.0 for _ in self.base_lrs]
        pct_remaining = (self.max_updates - self._step_count) / (self.max_updates - self.warmup_updates)
        return [base_lr * pct_remaining for base_lr in self.base_lrs]
