"""Per-step scalars read by the kernels from device memory.

A captured HIP graph replays fixed kernel arguments, so everything that changes from one optimizer
step to the next lives in one small device block that the host refreshes (stream-ordered, from a
pinned ring) before each step -- eager or replayed alike:

  [0:8)     uint64 RNG epoch: every dropout / HardConcrete kernel adds epoch * golden-ratio to its
            seed (common.h ``epoch_seed``), so a replay draws fresh noise and a step's backward
            regenerates exactly its forward's masks
  [8:12)    fp32 target sparsity of the Lagrangian regulariser (lightning.py:163-166, 267-273)
  [16:160)  DphAdamDyn: per-group lr / weight decay / betas / eps and the 1-based AdamW step
            (lightning.py:200-238 groups, LinearDecayLRScheduler lightning.py:22-44)

One block per device per process, never freed: the kernels' epoch pointer (dph_set_rng_epoch) refers
to it for the life of the process.
"""

import ctypes as C
import time
from typing import Dict, Optional, Sequence

import torch

from . import _lib
from ._lib import DphAdamDyn, call

BLOCK_BYTES = 256
OFF_EPOCH = 0
OFF_TARGET = 8
OFF_ADAM = 16
RING = 4

assert OFF_ADAM + C.sizeof(DphAdamDyn) <= BLOCK_BYTES


class StepScalars:
    def __init__(self, device: torch.device):
        self.device = device
        self.dev = torch.zeros(BLOCK_BYTES, dtype=torch.uint8, device=device)
        self.host = [torch.zeros(BLOCK_BYTES, dtype=torch.uint8).pin_memory() for _ in range(RING)]
        self.events: list = [None] * RING
        self.k = 0
        self.epoch = 0
        # host seconds spent blocked on the ring (a slot whose copy of RING steps ago has not run yet): with
        # graph replay the host runs at most RING steps ahead of the GPU, so a loop's host time minus this is the
        # host's own enqueue cost (bench.py host_enqueue_ms)
        self.wait_s = 0.0
        with torch.cuda.device(device):
            call("dph_set_rng_epoch", self.dev.data_ptr() + OFF_EPOCH)

    # device views -------------------------------------------------------------
    @property
    def target_sparsity(self) -> torch.Tensor:
        """0-d fp32 device view of the current target sparsity."""
        return self.dev[OFF_TARGET:OFF_TARGET + 4].view(torch.float32)[0]

    @property
    def adam_dyn_ptr(self) -> int:
        return self.dev.data_ptr() + OFF_ADAM

    # host -> device -----------------------------------------------------------
    def upload(self, *, target_sparsity: float = 0.0, adam_groups: Optional[Sequence[dict]] = None,
               adam_step: int = 0, advance_epoch: bool = True):
        """Write this step's scalars into the next pinned slot and copy it to the device block on the
        current stream (never inside a graph capture)."""
        if advance_epoch:
            self.epoch += 1
        i = self.k % RING
        self.k += 1
        if self.events[i] is not None and not self.events[i].query():
            t0 = time.perf_counter()
            self.events[i].synchronize()        # the copy that last read this pinned slot is done
            self.wait_s += time.perf_counter() - t0
        h = self.host[i]
        base = h.data_ptr()
        C.c_uint64.from_address(base + OFF_EPOCH).value = self.epoch & 0xFFFFFFFFFFFFFFFF
        C.c_float.from_address(base + OFF_TARGET).value = float(target_sparsity)
        dyn = DphAdamDyn.from_address(base + OFF_ADAM)
        for gi, g in enumerate(adam_groups or []):
            dyn.g[gi].lr = g["lr"]
            dyn.g[gi].weight_decay = g["weight_decay"]
            dyn.g[gi].beta1 = g["betas"][0]
            dyn.g[gi].beta2 = g["betas"][1]
            dyn.g[gi].eps = g["eps"]
        dyn.step = float(adam_step)
        self.dev.copy_(h, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.events[i] = ev


_BLOCKS: Dict[int, StepScalars] = {}


def step_scalars(device) -> StepScalars:
    """The process-wide block of ``device`` (created on first use)."""
    device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    blk = _BLOCKS.get(idx)
    if blk is None:
        blk = StepScalars(torch.device("cuda", idx))
        _BLOCKS[idx] = blk
    return blk
