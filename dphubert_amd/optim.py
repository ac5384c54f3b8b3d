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
from torch.autograd.graph import increment_version

from . import _lib
from ._lib import DphAdamGroup, DphTensorSlot, call, ptr

CHUNK = 8192   # must match optim.hip
SUMSQ_FLOATS = 1025   # DPH_SUMSQ_FLOATS (include/dphubert_hip.h)


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
        self._slot_key = None
        self._step = 0
        self._step_t = torch.zeros((), dtype=torch.float32)   # one counter shared by every param's state
        self.dyn_ptr = None          # device DphAdamDyn (stepstate.StepScalars) -> dph_adamw_step_dev

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
        self._sumsq = torch.zeros(SUMSQ_FLOATS, dtype=torch.float32, device=dev)   # [0] = ||g||^2, [1:] partials
        self._chunk_key = key

    def _slot_table(self, plist):
        """Upload the (param, grad, exp_avg, exp_avg_sq) pointer table when any pointer changed.
        With a GradReducer the gradients are fixed bucket views, so this runs once."""
        key = []
        for gi, p in plist:
            st = self.state[p]
            if len(st) == 0:
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] = self._step_t
            elif st.get("step") is not self._step_t:
                # loaded state (load_state_dict): adopt its step count, then share one counter
                self._step = max(self._step, int(st["step"]))
                self._step_t.fill_(self._step)
                st["step"] = self._step_t
            if p.grad is not None and not p.grad.is_contiguous():
                p.grad = p.grad.contiguous()
            if p.grad is not None and p.grad.dtype != torch.float32:
                raise TypeError("FusedAdamW expects fp32 gradients")
            key.append((p.data_ptr(), p.grad.data_ptr() if p.grad is not None else 0, st["exp_avg"].data_ptr(),
                        st["exp_avg_sq"].data_ptr(), p.numel(), gi))
        key = tuple(key)
        if key == self._slot_key:
            return
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("FusedAdamW: parameter/gradient storage changed inside a HIP graph capture")
        if self._event is not None:
            self._event.synchronize()     # previous H2D copy of the pinned table is done
        slots = (DphTensorSlot * len(plist)).from_address(self._pinned.data_ptr())
        for i, (pp, gp, ma, va, n, gi) in enumerate(key):
            slots[i].param, slots[i].grad, slots[i].exp_avg, slots[i].exp_avg_sq = pp, gp, ma, va
            slots[i].n = n
            slots[i].group = gi
        self._slots_dev.copy_(self._pinned, non_blocking=True)
        self._event = torch.cuda.Event()
        self._event.record()
        self._slot_key = key

    def begin_step(self) -> int:
        """Host half of a step: advance the step counter; returns the 1-based AdamW step that a
        device-resident DphAdamDyn must carry together with the current ``param_groups`` values."""
        self._step += 1
        self._step_t.fill_(self._step)
        self._opt_called = True       # what torch's LRScheduler checks for "optimizer.step() ran first"
        return self._step

    @torch.no_grad()
    def launch(self):
        """Device half of a step: clip + AdamW over every parameter (2 launches), stream-ordered and
        capturable.  Reads lr / step from ``self.dyn_ptr`` (a DphAdamDyn in device memory) when set,
        else from ``param_groups`` at launch time."""
        plist = self._params()
        if not plist:
            return
        self._ensure_chunks(plist)
        self._slot_table(plist)
        s = _lib.stream_ptr()
        clip = self.max_grad_norm is not None and self.max_grad_norm > 0
        if clip:
            call("dph_grad_sumsq", ptr(self._slots_dev), len(plist), ptr(self._cslot), ptr(self._cstart),
                 self._nchunks, ptr(self._sumsq), s)
        from . import ops
        ids = {id(p) for _, p in plist}
        # the bf16 GEMM images of the updated weights are written by the AdamW kernel itself (one pass over the
        # masters instead of a second cast launch re-reading all of them)
        dst, cast_done = ops.image_targets(ids)
        img = ops._table([(dst.get(id(p), 0),) for _, p in plist])
        groups = (DphAdamGroup * 4)()
        if self.dyn_ptr is None:
            for gi, g in enumerate(self.param_groups):
                groups[gi].lr = g["lr"]
                groups[gi].weight_decay = g["weight_decay"]
                groups[gi].beta1 = g["betas"][0]
                groups[gi].beta2 = g["betas"][1]
                groups[gi].eps = g["eps"]
        from .kernels import SPAN_HINT
        SPAN_HINT["adamw_params"] = sum(p.numel() for _, p in plist)   # bench.py's kernel table (bytes per launch)
        call("dph_adamw_step_img", ptr(self._slots_dev), len(plist), ptr(self._cslot), ptr(self._cstart),
             self._nchunks, self.dyn_ptr, groups, len(self.param_groups), self._step,
             ptr(self._sumsq) if clip else None, float(self.max_grad_norm or 0.0), ptr(img), s)
        # the kernel wrote the masters behind autograd's back: bump their version counters so every
        # cached bf16 GEMM image of them (ops.bf16_image & co.) is rebuilt before its next use
        increment_version([p for _, p in plist])
        # cast the images the kernel did not cover, re-transpose the W^T images, and move the cache keys to the
        # new versions
        ops.refresh_images(ids, cast_done)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if not self._params():
            return loss
        self.begin_step()
        self.launch()
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
