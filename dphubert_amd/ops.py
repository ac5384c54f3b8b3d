"""Autograd layer: one ``torch.autograd.Function`` per reference module.

Each Function's forward/backward is a fixed schedule of HIP kernels from
libdphubert_hip.so (through ``kernels``): no ATen math runs on the hot path,
only allocation (caching allocator), views and a few O(channels) glue ops.
The Functions are coarse (a whole EncoderLayer, the whole conv frontend, ...)
so that cross-op fusion is possible (GEMM epilogues carry bias, GELU,
HardConcrete masks, dropout, layer masks and residuals; LayerNorm backward
emits the residual-branch gradient and its bias column sums in the same
pass) and Python/autograd overhead stays at a few dozen nodes per step.

Reference semantics followed (file:line of seas2nada/DPHuBERT):
  FrontendFn           components.py:94-120, 158-185, 1071-1076
  FeatureProjectionFn  components.py:263-274, 968-984
  PosConvFn            components.py:319-333, 885-892
  EncoderLayerFn       components.py:379-436, 726-748, 814-857
  DistillProjLossFn    lightning.py:250-265, 116-139
  HardConcreteFn       hardconcrete.py:85-99
  ExpectedParamsFn     model.py:109-113 + get_num_params chain
"""

import contextlib
import math
import os
from typing import List, Optional, Sequence

import torch

from . import _lib
from . import kernels as K
from ._lib import call, ptr

BF16 = torch.bfloat16
F32 = torch.float32
LOSS_PARTIAL_FLOATS = 3072      # DPH_LOSS_PARTIAL_FLOATS (include/dphubert_hip.h)

HC_BETA = 2.0 / 3.0
HC_LIMIT_L = -0.1
HC_LIMIT_R = 1.1
HC_EPS = 1e-6
HC_BIAS = -HC_BETA * math.log(-HC_LIMIT_L / HC_LIMIT_R)


def _s():
    return _lib.stream_ptr()


def _ws_t(nbytes: int, dev):
    """Scratch tensor for a column-partial slab (inside an armed deferred_reductions call it is kept alive until
    the block's flush)."""
    t = torch.empty(max(int(nbytes), 4) // 4, dtype=F32, device=dev)
    keep = K.KEEP_WS[0]
    if keep is not None and K.ARMED[0]:
        keep.append(t)
    return t


def _ws(nbytes: int, dev):
    """Scratch for a column-partial slab, as (pointer, bytes) for the NEXT library call (stream-ordered caching
    allocator: the block is reused only by work queued after the kernel that consumes it -- inside a
    deferred_reductions block the slab is kept alive until the block's flush, which is then that consumer).  The
    tensor itself is released at once: no other allocation may come between this and the call that uses it (it
    could be handed the same block) -- hold a ``_ws_t`` tensor instead where one must."""
    t = _ws_t(nbytes, dev)
    return ptr(t), t.numel() * 4


def ln_ws(rows: int, D: int, dev):
    return _ws(_lib.lib().dph_layernorm_bwd_workspace(rows, D), dev)


def colsum_ws(rows: int, cols: int, dev):
    return _ws(_lib.lib().dph_colsum_workspace(rows, cols), dev)


def rb_ws(rows: int, cols: int, dev):
    """Workspace of the per-row-block column reductions (GELU-mask / branch backward): their fixed-order partial
    slab in deterministic mode (include/dphubert_hip.h dph_rowblock_workspace)."""
    return _ws(_lib.lib().dph_rowblock_workspace(rows, cols), dev)


# ---------------------------------------------------------------------------
# counter-based seeds (dropout / HardConcrete noise)
# ---------------------------------------------------------------------------
class SeedSource:
    """Per-process 64-bit seed stream; reseeded by ``torch.manual_seed``-style calls."""

    def __init__(self, seed: int = 2022):
        self.reset(seed)

    def reset(self, seed: int):
        self._state = (int(seed) * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        self._n = 0

    def next(self) -> int:
        self._n += 1
        z = (self._state + self._n * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        return z ^ (z >> 31)


SEEDS = SeedSource()


def manual_seed(seed: int):
    SEEDS.reset(seed)


# ---------------------------------------------------------------------------
# bf16 GEMM images of fp32 master weights (cached per parameter version)
# ---------------------------------------------------------------------------
def _version_key(ts):
    return tuple((id(t), t._version) for t in ts)


def bf16_image(*ts: torch.Tensor) -> torch.Tensor:
    """Concatenate fp32 tensors (along dim 0) into one bf16 image.

    The image is cached ON the first tensor object (attribute), keyed by the identity and
    version counter of every source tensor, so an optimizer step (in-place update bumps
    ``_version``) or a different parameter set always rebuilds it, and the cache dies with
    the parameter.
    """
    owner = ts[0]
    key = ("cat",) + _version_key(ts)
    hit = getattr(owner, "_dph_img", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    rows = sum(t.shape[0] for t in ts)
    out = torch.empty((rows,) + tuple(ts[0].shape[1:]), dtype=BF16, device=ts[0].device)
    off = 0
    for t in ts:
        n = t.numel()
        call("dph_cast_bf16", ptr(t.detach()), out.data_ptr() + off * 2, n, _s())
        off += n
    if hit is not None:
        _REFRESH.pop(id(hit[1]), None)
        _T_REFRESH.pop(id(hit[1]), None)
    owner._dph_img = (key, out)
    if all(t.requires_grad for t in ts):
        _REFRESH[id(out)] = (owner, ts, out)
    return out


# Images of trained weights are refreshed IN PLACE right after the optimizer step by two batched
# launches (refresh_images, called by FusedAdamW.launch): one cast of every registered image and
# one transpose of every registered W^T image, instead of ~85 + ~50 separate few-us launches spread
# over the next forward / backward.  The cache keys are moved to the new parameter versions, so the
# next bf16_image / t_image calls hit.
_REFRESH = {}       # id(image) -> (owner, sources, image)
_T_REFRESH = {}     # id(image) -> (image, transposed image)
_TABLES = {}        # device tables of the batched launches, keyed by their content


def _table(rows) -> torch.Tensor:
    key = tuple(rows)
    t = _TABLES.get(key)
    if t is None:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("image refresh table changed during graph capture")
        # kept for the life of the process: a captured graph reads the table by address
        t = torch.tensor([v for r in rows for v in r], dtype=torch.int64).to(torch.device("cuda"), non_blocking=False)
        _TABLES[key] = t
    return t


def image_targets(updated_ids):
    """Where the optimizer kernel can write the bf16 casts itself (dph_adamw_step_img): {id(param): address of
    its rows in a registered image} for the images whose sources are all in ``updated_ids``, and the ids of the
    images fully covered that way (a parameter feeding two images casts into the first; the second stays with
    refresh_images)."""
    dst, covered = {}, set()
    for _owner, ts, out in _REFRESH.values():
        if not all(id(t) in updated_ids for t in ts) or any(id(t) in dst for t in ts):
            continue
        off = 0
        for t in ts:
            dst[id(t)] = out.data_ptr() + off * 2
            off += t.numel()
        covered.add(id(out))
    return dst, covered


def refresh_images(updated_ids, cast_done=frozenset()) -> None:
    """Recast every registered image whose sources are all in ``updated_ids`` (ids of parameters
    the optimizer just wrote) -- except the images in ``cast_done`` (ids: the optimizer kernel cast them,
    image_targets) --, re-transpose their W^T images, re-copy the fp32 concatenations, and re-key the caches."""
    cats = [e for e in _CAT_REFRESH.values() if all(id(t) in updated_ids for t in e[1])]
    if cats:
        crows = []
        for _owner, ts, out in cats:
            off = 0
            for t in ts:
                crows.append((t.data_ptr(), out.data_ptr() + off * 4, t.numel()))
                off += t.numel()
        call("dph_copy_f32_multi", ptr(_table(crows)), len(crows), max(r[2] for r in crows), _s())
        for owner, ts, out in cats:
            owner._dph_cat = (("f32cat",) + _version_key(ts), out)
    ents = [e for e in _REFRESH.values() if all(id(t) in updated_ids for t in e[1])]
    if not ents:
        return
    rows = []
    for _owner, ts, out in ents:
        if id(out) in cast_done:
            continue
        off = 0
        for t in ts:
            rows.append((t.data_ptr(), out.data_ptr() + off * 2, t.numel()))
            off += t.numel()
    if rows:
        call("dph_cast_bf16_multi", ptr(_table(rows)), len(rows), _s())
    for owner, ts, out in ents:
        owner._dph_img = (("cat",) + _version_key(ts), out)
    trows = [(img.data_ptr(), tout.data_ptr(), img.shape[0], img.shape[1])
             for img, tout in (_T_REFRESH.get(id(e[2]), (None, None)) for e in ents) if img is not None]
    if trows:
        ttab = _table(trows)
        call("dph_transpose_bf16_multi", ptr(ttab), len(trows), _s())


_CAT_REFRESH = {}   # id(concatenation) -> (owner, sources, concatenation)


def f32_cat(*ts: torch.Tensor) -> torch.Tensor:
    """Concatenation of fp32 parameters (e.g. the q/k/v biases), cached like bf16_image and refreshed by
    the optimizer's batched image refresh (one dph_copy_f32_multi launch for all of them)."""
    owner = ts[0]
    key = ("f32cat",) + _version_key(ts)
    hit = getattr(owner, "_dph_cat", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    n = sum(t.numel() for t in ts)
    out = torch.empty(n, dtype=F32, device=ts[0].device)
    rows, off = [], 0
    for t in ts:
        rows.append((t.detach().data_ptr(), out.data_ptr() + off * 4, t.numel()))
        off += t.numel()
    if torch.cuda.is_current_stream_capturing():
        out.copy_(torch.cat([t.detach() for t in ts]))       # (tables are built outside captures)
    else:
        call("dph_copy_f32_multi", ptr(_table(rows)), len(rows), max(r[2] for r in rows), _s())
    if hit is not None:
        _CAT_REFRESH.pop(id(hit[1]), None)
    owner._dph_cat = (key, out)
    if all(t.requires_grad for t in ts):
        _CAT_REFRESH[id(out)] = (owner, ts, out)
    return out


def pad8(n: int) -> int:
    """Storage width of a channel / feature dimension: pruned students have ragged widths, the
    bf16 kernels read 16-B chunks, so rows are padded to a multiple of 8 with zero columns."""
    return (int(n) + 7) // 8 * 8


def conv_image(w: torch.Tensor, Op: Optional[int] = None, Cp: Optional[int] = None) -> torch.Tensor:
    """conv weight [O][C][k] fp32 -> bf16 [Op][k*Cp] (k-major, matches channels-last im2col rows;
    zero rows / channels for the 8-padding of pruned widths)."""
    O, C, kk = w.shape
    Op = Op or O
    Cp = Cp or C
    key = ("conv", Op, Cp) + _version_key((w,))
    hit = getattr(w, "_dph_img", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    out = torch.empty(Op, kk * Cp, dtype=BF16, device=w.device)
    call("dph_conv_weight_pack", ptr(w.detach()), ptr(out), O, C, kk, Op, Cp, _s())
    w._dph_img = (key, out)
    return out


def padded_image(w: torch.Tensor, rows_p: int, cols_p: int) -> torch.Tensor:
    """bf16 image of a 2-D fp32 weight zero-padded to [rows_p][cols_p] (pruned widths), cached
    like bf16_image; the padding glue is plain torch and runs once per optimizer step."""
    if tuple(w.shape) == (rows_p, cols_p):
        return bf16_image(w)
    key = ("pad", rows_p, cols_p) + _version_key((w,))
    hit = getattr(w, "_dph_img", None)
    if hit is not None and hit[0] == key:
        return hit[1]
    out = torch.zeros(rows_p, cols_p, dtype=BF16, device=w.device)
    out[:w.shape[0], :w.shape[1]] = w.detach().to(BF16)
    w._dph_img = (key, out)
    return out


# input-gradient GEMMs take the transposed weight image (k-contiguous B: ring kernels); DPH_DGRAD_T=0
# keeps the mn-contiguous B operand (register-staged kernel) for A/B timing
_DGRAD_T = os.environ.get("DPH_DGRAD_T", "1") != "0"
# strided-conv input gradients by output phase (no column gradient / col2im); DPH_PHASE_DGRAD=0 keeps
# the column path (A/B timing, tests of both)
_PHASE_DGRAD = os.environ.get("DPH_PHASE_DGRAD", "1") != "0"


def t_image(img: torch.Tensor) -> Optional[torch.Tensor]:
    """[C][R] transpose of a bf16 weight image [R][C], cached on the image tensor (an image is
    rebuilt whenever its fp32 master changes, so the transpose follows it); None when disabled or
    the widths are not multiples of 8."""
    if not _DGRAD_T or img.dim() != 2 or img.shape[0] % 8 or img.shape[1] % 8:
        return None
    hit = getattr(img, "_dph_t", None)
    if hit is not None:
        return hit
    out = torch.empty(img.shape[1], img.shape[0], dtype=BF16, device=img.device)
    call("dph_transpose_bf16", ptr(img), img.shape[0], img.shape[1], ptr(out), _s())
    img._dph_t = out
    if id(img) in _REFRESH:
        _T_REFRESH[id(img)] = (img, out)
    return out


def conv_frame_lengths(length: torch.Tensor, layers) -> torch.Tensor:
    """components.py:179-181 over every conv layer (L = max(0, floor((L - k) / s) + 1)) in one launch."""
    import ctypes
    n = len(layers)
    ks = (ctypes.c_int32 * n)(*[int(k) for _, k, _ in layers])
    ss = (ctypes.c_int32 * n)(*[int(s_) for _, _, s_ in layers])
    src = length.to(torch.int64).contiguous()
    out = torch.empty_like(src)
    call("dph_conv_lengths", ptr(src), ptr(out), src.numel(), n, ctypes.addressof(ks), ctypes.addressof(ss), _s())
    return out


def padded_vec(v: Optional[torch.Tensor], n_p: int) -> Optional[torch.Tensor]:
    """fp32 vector zero-padded to n_p (bias / mask of a pruned width); the same tensor if no padding."""
    if v is None or v.numel() == n_p:
        return v
    out = torch.zeros(n_p, dtype=v.dtype, device=v.device)
    out[:v.numel()] = v
    return out


class _ZeroArena:
    """Zero-filled fp32 slices carved from 4 MB chunks: one fill per chunk instead of one fill
    kernel per small gradient / accumulator buffer (~100 per step).  Slices are never reused
    (the offset only grows); a chunk is freed by the caching allocator once every slice is dead."""

    CHUNK = 1 << 20

    def __init__(self):
        self.buf = None
        self.off = 0

    def take(self, n: int, dev) -> torch.Tensor:
        n_al = (n + 63) // 64 * 64
        if n_al > self.CHUNK // 4:
            return torch.zeros(n, dtype=F32, device=dev)
        if self.buf is None or self.off + n_al > self.CHUNK or self.buf.device != torch.device(dev):
            self.buf = torch.zeros(self.CHUNK, dtype=F32, device=dev)
            self.off = 0
        t = self.buf[self.off:self.off + n]
        self.off += n_al
        return t


_ZEROS = _ZeroArena()


_ARENAS = []


def new_zero_arena() -> _ZeroArena:
    a = _ZeroArena()
    _ARENAS.append(a)
    return a


class private_zero_arena:
    """Route zeros_f32 to ``arena`` inside the block (work on a side stream must not share arena
    chunks whose zero fill sits on another stream)."""

    def __init__(self, arena: _ZeroArena):
        self.arena = arena

    def __enter__(self):
        global _ZEROS
        self.prev, _ZEROS = _ZEROS, self.arena
        return self.arena

    def __exit__(self, *exc):
        global _ZEROS
        _ZEROS = self.prev


def reset_zero_arena():
    """Start a fresh arena chunk on the next request (around a HIP-graph capture: slices handed out
    inside the capture must come from a chunk whose zero fill is itself part of the graph)."""
    for a in [_ZEROS] + _ARENAS:
        a.buf = None
        a.off = 0


def zeros_f32(shape, dev) -> torch.Tensor:
    """Zero-filled fp32 tensor (small ones come from the arena, no fill kernel of their own)."""
    if isinstance(shape, int):
        shape = (shape,)
    n = 1
    for d in shape:
        n *= d
    return _ZEROS.take(n, dev).view(shape)


def _zeros(n, like_device, dtype=F32):
    return zeros_f32(n, like_device) if dtype == F32 else torch.zeros(n, dtype=dtype, device=like_device)


# ---------------------------------------------------------------------------
# weight-gradient GEMMs on a side stream (Trainer: wgrad_overlap)
# ---------------------------------------------------------------------------
# A layer's weight gradients feed nothing else in the backward (only the optimizer, or the bucket's
# all-reduce), so they run on a second HIP stream, concurrently with the input-gradient chain: their
# blocks fill the CUs the chain's N = 768 GEMM rounds, attention tails and latency-bound LayerNorm /
# reduction launches leave idle (the backward counterpart of the teacher-forward stream).  Only
# gradients written into bucket sinks move (autograd never reads them); the backward's exit joins the
# side stream, and GradOut.done() joins it before a bucket's collective is launched.
_WGRAD_SIDE = [None]
# which weight gradients move: "all" (encoder layers + conv frontend) or "conv" (DPH_WGRAD_SCOPE)
_WGRAD_SCOPE = os.environ.get("DPH_WGRAD_SCOPE", "conv")


class wgrad_overlap:
    """Inside the block (one backward), sink-bound weight-gradient GEMMs launch on ``stream``; GEMMs of the
    main stream take one tile per block meanwhile (a persistent grid would wait for CUs the side stream
    holds).  Exit: the main stream waits for the side stream."""

    def __init__(self, stream):
        self.stream = stream
        share = _WGRAD_SCOPE == "all" and os.environ.get("DPH_WGRAD_PERSIST", "0") != "1"
        self.shared = K.shared_gpu() if share else contextlib.nullcontext()

    def __enter__(self):
        if self.stream is not None:
            self.prev, _WGRAD_SIDE[0] = _WGRAD_SIDE[0], self.stream
            self.shared.__enter__()
        return self

    def __exit__(self, *exc):
        if self.stream is not None:
            _WGRAD_SIDE[0] = self.prev
            self.shared.__exit__(*exc)
            torch.cuda.current_stream().wait_stream(self.stream)


class wgrad_side:
    """Run the block on the weight-gradient side stream when one is active and ``enable`` (the output is a
    bucket sink): forked from the main stream, and every tensor in ``inputs`` marked as used by the side
    stream (the caching allocator then keeps it until the side stream's work is done)."""

    def __init__(self, *inputs, enable: bool = True, scope: str = "enc"):
        self.inputs = inputs
        self.side = _WGRAD_SIDE[0] if (enable and (_WGRAD_SCOPE == "all" or scope == _WGRAD_SCOPE)) else None

    def __enter__(self):
        if self.side is not None:
            self.side.wait_stream(torch.cuda.current_stream())
            self.ctx = torch.cuda.stream(self.side)
            self.ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.side is not None:
            self.ctx.__exit__(*exc)
            for t in self.inputs:
                if t is not None:
                    t.record_stream(self.side)


# ---------------------------------------------------------------------------
# grouped encoder-layer weight gradients (Trainer: wgrad_group)
# ---------------------------------------------------------------------------
# One layer's weight-gradient GEMMs (dW = dY^T X, K = the B*T frames) have few output tiles (768 x 768: 18 tiles of
# 128 x 256), so each needs split-K slices, their fp32 slab and a reduce launch to fill 256 CUs.  Inside a
# grouped_wgrads block the bucket-sink ones are queued per shape and launched ``group`` layers at a time as ONE
# grouped GEMM (dph_gemm_grouped: problem z = layer), which fills the CUs with whole-K blocks.  The queued
# gradients' parameters are held back from the reducer (p._dph_hold) until their group lands, so a bucket's
# collective still starts only after all its gradients are written; the queue keeps dY / X alive until then.
_WGRAD_DEFER = [None]


class grouped_wgrads:
    """Queue the encoder layers' bucket-sink weight-gradient GEMMs of one backward and launch them ``group``
    layers at a time (exit flushes the rest).  ``group`` <= 1: no-op."""

    def __init__(self, group: int = 6):
        self.group = min(int(group), _lib.GEMM_GROUP_MAX)
        self.queues = {}

    def __enter__(self):
        if self.group > 1:
            self.prev, _WGRAD_DEFER[0] = _WGRAD_DEFER[0], self
        return self

    def __exit__(self, exc_type, *exc):
        if self.group > 1:
            _WGRAD_DEFER[0] = self.prev
            if exc_type is None:
                self.flush()
            else:
                for items in self.queues.values():
                    for *_, params, _post in items:
                        for p in params:
                            p._dph_hold = False
                self.queues = {}

    def add(self, dy, x, dw, params, post=None):
        key = (tuple(dy.shape), tuple(x.shape), dy.device, K.ROLE[0])
        items = self.queues.setdefault(key, [])
        for p in params:
            p._dph_hold = True
        items.append((dy, x, dw, params, post))
        if len(items) >= self.group:
            self._flush(key)

    def _flush(self, key):
        items = self.queues.pop(key)
        # a group whose gradients nothing else in the backward reads (no post(): the FFN2 group's feeds the FFN
        # mask gradient the HardConcrete backward consumes) may run on the weight-gradient side stream
        # (DPH_WGRAD_STREAM=1 with DPH_WGRAD_SCOPE=group / all), beside the rest of the backward
        side_ok = all(post is None for *_, post in items)
        ins = [t for dy, x, *_ in items for t in (dy, x)]
        with wgrad_side(*ins, enable=side_ok, scope="group"), K.role(key[3]):
            ws = K.linear_wgrad_grouped([(dy, x, dw) for dy, x, dw, _, _ in items], accumulate=True)
            del ws
            for *_, params, post in items:
                if post is not None:
                    post()       # reads the landed weight gradient (stream-ordered after the grouped launch)
                for p in params:
                    p._dph_hold = False
                    p._dph_sink_ready(p)

    def flush(self):
        for key in list(self.queues):
            self._flush(key)


def _flush_wgrads_hook(grad):
    q = _WGRAD_DEFER[0]
    if q is not None:
        q.flush()
    r = _RED_DEFER[0]
    if r is not None:
        r.close()
    return None


# ---------------------------------------------------------------------------
# deferred column reductions (Trainer: one backward = one deferred_reductions block)
# ---------------------------------------------------------------------------
# In deterministic mode each bias / LayerNorm-affine gradient is a per-block partial slab summed in a fixed order
# by its own small grid (~4-5 us each, ~50 per encoder backward).  Inside a deferred_reductions block the ones whose
# outputs are bucket-sink gradients (nothing in the backward reads them) are queued by the library
# (dph_defer_reductions) and launched together when the encoder backward ends (the flush of the encoder-input hook,
# next to the grouped weight gradients) -- one grid per 96 reductions, bitwise the same sums.  Their parameters are
# held back from the reducer until then, and their slabs kept alive.
_RED_DEFER = [None]


class deferred_reductions:
    """Queue the sink-bound column reductions of one backward (see above); close() / exit flush them."""

    def __init__(self, enable: bool = True):
        self.enable = bool(enable) and os.environ.get("DPH_DEFER_RED", "1") != "0" and _lib.deterministic()
        self.keep, self.pending = [], []
        self.open = False

    def __enter__(self):
        if self.enable:
            left = int(_lib.lib().dph_deferred_reductions())
            if left:
                raise RuntimeError(f"deferred_reductions: {left} column reductions left queued by an earlier block")
            self.prev, _RED_DEFER[0] = _RED_DEFER[0], self
            self.prev_keep, K.KEEP_WS[0] = K.KEEP_WS[0], self.keep
            self.open = True
        return self

    def arm(self, go, ok: bool):
        """Context of one library call whose column reductions may be queued (``ok``: all their outputs are
        bucket sinks)."""
        return _Armed(self if (self.open and ok) else None, go)

    def close(self):
        """Launch the queued reductions, then release their parameters to the reducer; later calls run as usual."""
        if not self.open:
            return
        self.open = False
        K.KEEP_WS[0] = self.prev_keep
        call("dph_flush_reductions", _s())
        pend, self.pending = self.pending, []
        for p in pend:
            p._dph_defer_hold = False
        for p in pend:
            p._dph_sink_ready(p)
        self.keep = []

    def __exit__(self, exc_type, *exc):
        if self.enable:
            _RED_DEFER[0] = self.prev
            if exc_type is None:
                self.close()
            else:
                # the block failed (e.g. a graph capture that raised): the queued problems refer to slabs this block
                # no longer keeps and to sinks whose step is abandoned -- drop them unlaunched, so that no later flush
                # adds them into the next step's gradients
                self.open = False
                K.KEEP_WS[0] = self.prev_keep
                K.ARMED[0] = False
                _lib.lib().dph_defer_reductions(0)
                _lib.lib().dph_discard_reductions()
                for p in self.pending:
                    p._dph_defer_hold = False
                self.pending, self.keep = [], []


class _Armed:
    def __init__(self, scope, go):
        self.scope, self.go = scope, go

    def __enter__(self):
        if self.scope is not None:
            L = _lib.lib()
            L.dph_defer_reductions(1)
            K.ARMED[0] = True
            self.pushed0, self.keep0 = int(L.dph_reductions_pushed()), len(self.scope.keep)
            self.go.deferred = self.scope
        return self

    def __exit__(self, *exc):
        if self.scope is not None:
            L = _lib.lib()
            L.dph_defer_reductions(0)
            K.ARMED[0] = False
            if int(L.dph_reductions_pushed()) == self.pushed0:
                # nothing queued by this call (its reductions ran immediately): its slabs need not outlive it
                del self.scope.keep[self.keep0:]


def _defer_red(go, *outs_direct):
    """Arm reduction deferral for the next library call when a deferred_reductions block is open and every output
    of its column reductions is a bucket sink (``outs_direct``: the GradOut ``direct`` flags)."""
    r = _RED_DEFER[0]
    if r is None:
        return _Armed(None, go)
    return r.arm(go, all(outs_direct))


def mark_encoder_input(x: torch.Tensor) -> torch.Tensor:
    """Hook the first encoder layer's input (Transformer._preprocess's output): its gradient is computed when the
    encoder backward ends, and the hook launches the layer weight gradients still queued in a grouped_wgrads block
    right then -- so every encoder bucket's collective is issued before the frontend backward (pos-conv, feature
    projection, conv stack) instead of at the end of the whole backward when the group size does not divide the
    layer count."""
    if x.requires_grad:
        x.register_hook(_flush_wgrads_hook)
    return x


def _layer_wgrad(dy, x, dw, direct, params, post=None, **kw):
    """An encoder layer's weight gradient: queued in the active grouped_wgrads block when it goes straight
    into the bucket (``direct``) at the operands' full width, else launched now (on the wgrad side stream
    when one is active).  ``post()`` runs once the gradient has landed (after its launch, or after the grouped
    launch that carries it)."""
    q = _WGRAD_DEFER[0]
    full = tuple(dw.shape) == (dy.shape[1], x.shape[1]) and kw.get("n_out", 0) in (0, dy.shape[1]) and \
        kw.get("k_in", 0) in (0, x.shape[1])
    if q is not None and direct and full:
        q.add(dy, x, dw, params, post)
        return None
    with wgrad_side(dy, x, enable=direct):
        ws = K.linear_wgrad(dy, x, dw, accumulate=direct, **kw)
    if post is not None:
        post()
    return ws


def _bucket_fresh(p) -> bool:
    """The gradient bucket behind ``p``'s sink holds this micro-batch's gradient alone (zeroed at its start)."""
    red = getattr(getattr(p, "_dph_sink_ready", None), "__self__", None)
    return red is not None and bool(getattr(red, "fresh", False))


# FFN intermediate-mask gradient from the FFN2 weight gradient (dph_colprod: sum_o W2[o][n] dW2[o][n] / mask_n)
# instead of re-reading the forward's f in the FFN2 input-gradient epilogue; DPH_FFN_COLPROD=0 keeps the epilogue
_FFN_COLPROD = os.environ.get("DPH_FFN_COLPROD", "1") != "0"
_TEACHER_OU = os.environ.get("DPH_TEACHER_OU", "0") == "1"   # A/B: the no-grad attention forward writes o_u / lse


# ---------------------------------------------------------------------------
# gradient sinks: weight gradients written straight into the data-parallel buckets
# ---------------------------------------------------------------------------
def _sink_view(params) -> Optional[torch.Tensor]:
    """Bucket storage of ``params`` (back-to-back, as one tensor over the concatenated rows) when
    a GradReducer has armed sinks on all of them, else None (see ddp.GradReducer.prepare)."""
    sinks = [getattr(p, "_dph_sink", None) if p is not None else None for p in params]
    if any(s is None for s in sinks):
        return None
    flat, off = sinks[0][0], sinks[0][1]
    n = 0
    for (f, o, _), p in zip(sinks, params):
        if f is not flat or o != off + n:
            return None
        n += p.numel()
    rows = sum(p.shape[0] for p in params)
    return flat[off:off + n].view((rows,) + tuple(params[0].shape[1:]))


class GradOut:
    """Hands out gradient buffers inside a Function's backward.

    ``buf(*params)`` returns ``(tensor, direct)``: with ``direct`` the tensor IS the parameters'
    bucket storage (kernels must accumulate into it, and autograd gets ``None`` for them, so no
    zero-fill / AccumulateGrad add ever runs for these gradients); otherwise a fresh fp32 tensor
    (zero-filled when ``zero``).  ``ret(*params)`` is what backward returns for the same params,
    and ``done()`` tells the reducer those gradients are complete (stream-ordered).
    """

    def __init__(self, dev):
        self.dev = dev
        self.sunk = set()
        self.sunk_params = []
        self.bufs = {}
        self.deferred = None     # the deferred_reductions block that queued reductions into these buffers

    def buf(self, *params, zero: bool = True):
        t = _sink_view(params)
        direct = t is not None
        if direct:
            self.sunk.update(id(p) for p in params)
            self.sunk_params.extend(params)
        else:
            rows = sum(p.shape[0] for p in params)
            shape = (rows,) + tuple(params[0].shape[1:])
            t = zeros_f32(shape, self.dev) if zero else torch.empty(shape, dtype=F32, device=self.dev)
        off = 0
        for p in params:
            self.bufs[id(p)] = t[off:off + p.shape[0]]
            off += p.shape[0]
        return t, direct

    def ret(self, p):
        if p is None or id(p) in self.sunk:
            return None
        return self.bufs.get(id(p))

    def done(self):
        side = _WGRAD_SIDE[0]
        if side is not None and self.sunk_params:
            red = getattr(self.sunk_params[0]._dph_sink_ready, "__self__", None)
            if red is not None and red.enabled and red.sync:
                torch.cuda.current_stream().wait_stream(side)   # the bucket's collective reads these gradients
        d = self.deferred
        if d is not None and d.open:
            # complete only once the queued reductions are flushed: held from the reducer until then (the autograd
            # post-accumulate hook of these parameters fires right after this backward returns and would otherwise
            # count them ready -- a bucket holding only such parameters was all-reduced before the flush wrote
            # them, tests/test_ddp_trainer_gpu.py with 8 MB buckets)
            for p in self.sunk_params:
                p._dph_defer_hold = True
            d.pending.extend(self.sunk_params)
            return
        for p in self.sunk_params:
            p._dph_sink_ready(p)


def _dev(t):
    return t.device


# k_proj.bias gradient: mathematically exactly zero (below), so it is not computed by default.  The reference's
# autograd evaluates it in floating point -- rounding noise of a sum that cancels to 0 -- and AdamW turns that noise
# into +-lr steps, so a reference-trained checkpoint's k_proj.bias drifts where ours stays put (the model output is
# unchanged either way).  DPH_KBIAS_GRAD=1 computes the column sum of dK as the reference does (checkpoint-matching
# runs; its values are noise and are not parity-pinned).
_KBIAS_GRAD = os.environ.get("DPH_KBIAS_GRAD", "0") == "1"
# DPH_ATTN_QV=0: the q / v bias gradients as a separate column-sum pass over dqkv (dph_colsum3) instead of inside the
# attention backward (A/B timing)
_ATTN_QV = os.environ.get("DPH_ATTN_QV", "1") != "0"


def _qkv_bias_grad(dqkv, dbqkv, M, dev):
    """q / v bias gradients (+=) as column sums of dQ / dV; the k bias gradient is exactly zero (softmax shift
    invariance, components.py:411-417) and its slot of the fused [3*Dh] buffer is left untouched (zeroed)."""
    Dh = dqkv.shape[1] // 3
    base = dbqkv.data_ptr()
    call("dph_colsum3", ptr(dqkv), base, base + 4 * Dh if _KBIAS_GRAD else None, base + 8 * Dh, M, Dh,
         *colsum_ws(M, 3 * Dh, dev), _s())


# ---------------------------------------------------------------------------
# HardConcrete sampling (training mode)
# ---------------------------------------------------------------------------
class HardConcreteFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, log_alpha, u_in):
        n = log_alpha.numel()
        mask = torch.empty_like(log_alpha)
        u = torch.empty_like(log_alpha) if u_in is None else u_in
        call("dph_hc_sample_fwd", ptr(log_alpha), ptr(u_in), None if u_in is not None else ptr(u), ptr(mask), n,
             SEEDS.next(), HC_BETA, HC_LIMIT_L, HC_LIMIT_R, HC_EPS, _s())
        ctx.save_for_backward(log_alpha, u)
        return mask

    @staticmethod
    def backward(ctx, dmask):
        la, u = ctx.saved_tensors
        dla = zeros_f32(tuple(la.shape), la.device)
        call("dph_hc_sample_bwd", ptr(la), ptr(u), ptr(dmask.contiguous()), ptr(dla), la.numel(), HC_BETA,
             HC_LIMIT_L, HC_LIMIT_R, _s())
        return dla, None


class RegLossFn(torch.autograd.Function):
    """loss = distill + lambda1*(es - t) + lambda2*(es - t)^2 with es = 1 - num/orig (lightning.py:221-229):
    one single-thread kernel forward (dph_reg_loss_fwd) and one backward, instead of ~10 + ~12 one-element
    ATen launches.  Returns (loss, loss_reg, expected_sparsity) as 0-d device tensors; ``target`` is a
    0-d device tensor (the HIP-graph step block) or a float."""

    @staticmethod
    def forward(ctx, distill, num, lambda1, lambda2, target, orig: float):
        dev = distill.device
        out = torch.empty(3, dtype=F32, device=dev)
        tdev = target if torch.is_tensor(target) else None
        tval = 0.0 if tdev is not None else float(target)
        for t in (distill, num, lambda1, lambda2) + ((tdev,) if tdev is not None else ()):
            if t.dtype != F32 or t.numel() != 1 or not t.is_contiguous():
                raise ValueError("RegLossFn: fp32 scalar tensors expected")
        call("dph_reg_loss_fwd", ptr(distill), ptr(num), ptr(lambda1), ptr(lambda2), ptr(tdev), tval, float(orig),
             ptr(out), _s())
        ctx.save_for_backward(num, lambda1, lambda2, *((tdev,) if tdev is not None else ()))
        ctx.tval, ctx.orig, ctx.has_t = tval, float(orig), tdev is not None
        ctx.lambdas = (lambda1, lambda2)      # the Parameters themselves (their gradient sinks)
        return out[0], out[1], out[2]

    @staticmethod
    def backward(ctx, g_loss, g_reg, g_es):
        saved = ctx.saved_tensors
        num, l1, l2 = saved[:3]
        tdev = saved[3] if ctx.has_t else None
        grads = torch.empty(3, dtype=F32, device=num.device)
        gs = [g.contiguous() if g is not None else None for g in (g_loss, g_reg, g_es)]
        sinks = [getattr(p, "_dph_sink", None) for p in ctx.lambdas]
        direct = all(sk is not None for sk in sinks)
        sp = [sk[0].data_ptr() + sk[1] * 4 for sk in sinks] if direct else [None, None]
        call("dph_reg_loss_bwd", ptr(gs[0]), ptr(gs[1]), ptr(gs[2]), ptr(num), ptr(l1), ptr(l2), ptr(tdev), ctx.tval,
             ctx.orig, ptr(grads), sp[0], sp[1], _s())
        if direct:
            for p in ctx.lambdas:
                p._dph_sink_ready(p)
            return g_loss, grads[0].view(num.shape), None, None, None, None
        return g_loss, grads[0].view(num.shape), grads[1].view(l1.shape), grads[2].view(l2.shape), None, None


class HardConcreteBank:
    """Every HardConcrete gate of one model (in the order of its expected-size polynomial table), sampled by
    ONE launch per step and differentiated by ONE launch, together with the expected #params (model.py:109-113)
    so that both gradients of a log_alpha land in one backward node (no AccumulateGrad adds)."""

    def __init__(self, mods, table: "ExpectedParamsTable"):
        self.mods = list(mods)
        self.table = table
        self.sizes = [m.log_alpha.numel() for m in self.mods]
        # each gate's slice of the flat u / mask / gradient buffers starts 16-B aligned: the masks are read as
        # float4 column vectors by the GEMM register epilogues (a misaligned colmask sends a GEMM off the
        # ping-pong kernels)
        self.offsets, o = [], 0
        for n in self.sizes:
            self.offsets.append(o)
            o += (n + 3) // 4 * 4
        self.total = max(o, 1)
        dev = table.offsets.device if table is not None else "cpu"
        self.offsets_dev = torch.tensor(self.offsets or [0], dtype=torch.int64, device=dev)

    def noise(self, m):
        """Injected u of a gate (HardConcrete.set_noise) as a device fp32 tensor (converted once), or None."""
        u = m._noise
        if u is None:
            return None
        hit = getattr(m, "_noise_dev", None)
        if hit is not None and hit[0] is u:
            return hit[1]
        d = u.to(m.log_alpha.device, torch.float32).contiguous()
        m._noise_dev = (u, d)
        return d


def _hc_entries(rows):
    arr = (_lib.DphHcEntry * len(rows))()
    for e, (la, uin, dm, dla, n, off) in zip(arr, rows):
        e.log_alpha, e.u_in, e.dmask, e.dlog_alpha, e.n, e.offset = la, uin, dm, dla, n, off
    return arr


class HardConcreteBankFn(torch.autograd.Function):
    """forward(bank, *log_alphas) -> (*masks, expected #params); backward: one poly-gradient launch + one gate
    launch, accumulating straight into the data-parallel buckets when their sinks are armed."""

    @staticmethod
    def forward(ctx, bank: HardConcreteBank, *las):
        dev = las[0].device
        u = torch.empty(bank.total, dtype=F32, device=dev)
        masks = torch.empty(bank.total, dtype=F32, device=dev)
        noise = [bank.noise(m) for m in bank.mods]
        rows = [(la.data_ptr(), ptr(nz), None, None, n, off) for la, nz, n, off in
                zip(las, noise, bank.sizes, bank.offsets)]
        call("dph_hc_bank_fwd", _hc_entries(rows), len(rows), ptr(u), ptr(masks), SEEDS.next(), HC_BETA, HC_LIMIT_L,
             HC_LIMIT_R, HC_EPS, _s())
        table = bank.table
        l0 = torch.empty(len(las), dtype=F32, device=dev)
        num = torch.empty((), dtype=F32, device=dev)
        call("dph_expected_params_fwd", ptr(table.ptr_table(las)), ptr(table.sizes), len(las), ptr(table.coef),
             ptr(table.idx), table.n_terms, table.constant, HC_BIAS, ptr(l0), ptr(num), _s())
        ctx.bank = bank
        ctx.save_for_backward(u, l0, *las)
        return tuple(masks[o:o + n].view_as(la) for la, n, o in zip(las, bank.sizes, bank.offsets)) + (num,)

    @staticmethod
    def backward(ctx, *grads):
        bank = ctx.bank
        u, l0, *las = ctx.saved_tensors
        dmasks, dnum = grads[:-1], grads[-1]
        dev = u.device
        table = bank.table
        sinks = [getattr(la, "_dph_sink", None) for la in las]
        direct = all(sk is not None for sk in sinks) and all(sk[0] is sinks[0][0] for sk in sinks)
        if direct:
            gflat = sinks[0][0]
            goff = _table([(sk[1],) for sk in sinks])
            dst = [gflat.data_ptr() + 4 * sk[1] for sk in sinks]
        else:
            gflat = zeros_f32(bank.total, dev)
            goff = bank.offsets_dev
            dst = [gflat.data_ptr() + 4 * o for o in bank.offsets]
        if dnum is not None:
            call("dph_expected_params_bwd", ptr(table.ptr_table(las)), ptr(gflat), ptr(goff), ptr(table.sizes),
                 len(las), ptr(table.coef), ptr(table.idx), table.n_terms, ptr(l0), ptr(dnum.contiguous()), HC_BIAS,
                 _s())
        keep = [dm.contiguous() if dm is not None else None for dm in dmasks]
        rows = [(la.data_ptr(), None, ptr(dm), d, n, off) for la, dm, d, n, off in
                zip(las, keep, dst, bank.sizes, bank.offsets)]
        if any(dm is not None for dm in keep):
            call("dph_hc_bank_bwd", _hc_entries(rows), len(rows), ptr(u), HC_BETA, HC_LIMIT_L, HC_LIMIT_R, _s())
        if direct:
            for la in las:
                la._dph_sink_ready(la)
            return (None,) * (1 + len(las))
        return (None,) + tuple(gflat[o:o + n].view_as(la) for la, n, o in zip(las, bank.sizes, bank.offsets))


# ---------------------------------------------------------------------------
# Expected number of parameters (differentiable, from l0 norms)
# ---------------------------------------------------------------------------
class ExpectedParamsTable:
    """Polynomial term table, built once per model config (see wav2vec2/model.py)."""

    def __init__(self, terms, constant, sizes, device):
        self.n_terms = len(terms)
        self.constant = float(constant)
        coef = [c for c, _ in terms] or [0.0]
        idx = []
        for _, ix in terms:
            ix = list(ix) + [-1] * (3 - len(ix))
            idx.extend(ix)
        if not idx:
            idx = [-1, -1, -1]
        self.coef = torch.tensor(coef, dtype=torch.float64, device=device)
        self.idx = torch.tensor(idx, dtype=torch.int32, device=device)
        self.sizes_list = [int(s) for s in sizes]
        self.sizes = torch.tensor(self.sizes_list or [0], dtype=torch.int64, device=device)
        offs = [0]
        for s in self.sizes_list:
            offs.append(offs[-1] + s)
        self.offsets = torch.tensor(offs[:-1] or [0], dtype=torch.int64, device=device)
        self.total = offs[-1]
        self._ptr_key = None
        self._ptrs = None

    def ptr_table(self, las):
        key = tuple(t.data_ptr() for t in las)
        if key != self._ptr_key:
            self._ptrs = torch.tensor(list(key) or [0], dtype=torch.int64, device=las[0].device if las else "cuda")
            self._ptr_key = key
        return self._ptrs


class ExpectedParamsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, table: ExpectedParamsTable, *las):
        dev = las[0].device if las else table.coef.device
        l0 = torch.empty(max(len(las), 1), dtype=F32, device=dev)
        out = torch.empty((), dtype=F32, device=dev)
        pt = table.ptr_table(las) if las else None
        call("dph_expected_params_fwd", ptr(pt), ptr(table.sizes), len(las), ptr(table.coef), ptr(table.idx),
             table.n_terms, table.constant, HC_BIAS, ptr(l0), ptr(out), _s())
        ctx.table = table
        ctx.save_for_backward(l0, *las)
        return out

    @staticmethod
    def backward(ctx, dout):
        l0, *las = ctx.saved_tensors
        table = ctx.table
        if not las:
            return (None,)
        g = zeros_f32(table.total, l0.device)
        call("dph_expected_params_bwd", ptr(table.ptr_table(las)), ptr(g), ptr(table.offsets), ptr(table.sizes),
             len(las), ptr(table.coef), ptr(table.idx), table.n_terms, ptr(l0), ptr(dout.contiguous()), HC_BIAS, _s())
        grads = []
        for off, n, la in zip(_offs(table), table.sizes_list, las):
            grads.append(g[off: off + n].view_as(la))
        return (None, *grads)


def _offs(table):
    out, o = [], 0
    for s in table.sizes_list:
        out.append(o)
        o += s
    return out


# ---------------------------------------------------------------------------
# Conv frontend (group_norm extractor)
# ---------------------------------------------------------------------------
class FrontendCfg:
    def __init__(self, layers, B, S, need_grad):
        self.layers = layers   # list of (out_c, k, s)
        self.B = B
        self.S = S
        self.need_grad = need_grad


def conv_lengths(S: int, layers) -> List[int]:
    out = []
    L = S
    for (_, k, s) in layers:
        L = max((L - k) // s + 1, 0)
        out.append(L)
    return out


def conv_dgrad_phases(dz: torch.Tensor, wt: torch.Tensor, B: int, Lout: int, Lin: int, O: int, Cin: int, k: int,
                      s: int, z_pre: Optional[torch.Tensor] = None, cm: Optional[torch.Tensor] = None,
                      dmask: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
    """Input gradient of a strided conv layer WITHOUT the [B*Lout][k*Cin] column gradient and its
    col2im pass: d_in[b][t'] = sum_{s*t + j = t'} dz[b][t] @ W_j, split by output phase (t' even /
    odd) into GEMMs that write d_in rows in place (components.py:107 conv backward).  With z_pre
    the previous layer's GELU'/mask backward runs in the GEMM epilogue (out = d*mask*GELU'(z_pre),
    dmask += d*GELU(z_pre)).  s = 2 and k in (2, 3) (every wav2vec2 / HuBERT conv1-6); returns None
    for other geometries (caller keeps the column path).  wt: transposed conv image [k*Cin][O]."""
    if s != 2 or k not in (2, 3) or Lout < 1 or Lin < 2 * Lout + k - 2:
        return None
    dev = dz.device
    d = torch.empty(B * Lin, Cin, dtype=BF16, device=dev)
    zflat = z_pre.view(-1) if z_pre is not None else None

    def gemm(A, Bm, coff, c_rpb, M, N, Kd, colmask=None, caux=None):
        kw = {}
        if z_pre is not None:
            kw = dict(act=K.ACT_GELU_BWD, aux_in=zflat[coff:], colmask=colmask, colsum_aux=caux)
        K.gemm(A, Bm, K.mat(d, 2 * Cin if c_rpb > 1 else Cin, rows_per_batch=c_rpb, batch_stride=Lin * Cin,
                            offset=coff), M, N, Kd, a_kcontig=True, b_kcontig=True, **kw)

    if k == 2:
        # t' = 2t + j: one GEMM over both taps, N = 2*Cin (the [W_0^T; W_1^T] rows of wt)
        cm2 = torch.cat([cm, cm]) if (z_pre is not None and cm is not None) else None
        dm2 = zeros_f32(2 * Cin, dev) if (z_pre is not None and dmask is not None) else None
        gemm(K.mat(dz, O), K.dense(wt), 0, Lout, B * Lout, 2 * Cin, O, cm2, dm2)
        if dm2 is not None:
            dmask += dm2[:Cin] + dm2[Cin:]
        if Lin > 2 * Lout:
            d.view(B, Lin, Cin)[:, 2 * Lout:].zero_()
        return d
    # k == 3: odd rows 2m+1 <- dz[m] W_1; interior even rows 2m (1 <= m < Lout) <- [dz[m-1], dz[m]] @
    # [W_2; W_0] (K = 2*O over two consecutive dz rows); edge rows 0 <- dz[0] W_0, 2*Lout <- dz[Lout-1] W_2
    gemm(K.mat(dz, O), K.mat(wt, O, offset=Cin * O), Cin, Lout, B * Lout, Cin, O, cm, dmask)
    if Lout > 1:
        weven = torch.cat([wt[2 * Cin:3 * Cin], wt[:Cin]], dim=1)
        gemm(K.mat(dz, O, rows_per_batch=Lout - 1, batch_stride=Lout * O), K.dense(weven), 2 * Cin, Lout - 1,
             B * (Lout - 1), Cin, 2 * O, cm, dmask)
    # the two edge-row GEMMs (B rows each) in ONE launch: grid batch z = 0 / 1 picks dz row 0 / Lout - 1, tap
    # W_0 / W_2 and output row 0 / 2 Lout (the z offsets), aux_in following the C layout
    kw = {}
    if z_pre is not None:
        kw = dict(act=K.ACT_GELU_BWD, aux_in=zflat, colmask=cm, colsum_aux=dmask)
    K.gemm(K.mat(dz, O, rows_per_batch=1, batch_stride=Lout * O, z_inner=(Lout - 1) * O),
           K.mat(wt, O, z_inner=2 * Cin * O),
           K.mat(d, Cin, rows_per_batch=1, batch_stride=Lin * Cin, z_inner=2 * Lout * Cin), B, Cin, O,
           a_kcontig=True, b_kcontig=True, batch=2, **kw)
    if Lin > 2 * Lout + 1:
        d.view(B, Lin, Cin)[:, 2 * Lout + 1:].zero_()
    return d


class FrontendFn(torch.autograd.Function):
    """wave (B,S) fp32 -> channels-last features (B*T, C) bf16 (x dummy_weight).

    inputs: wave, dummy_weight, gn_w, gn_b, then per layer i: conv weight, mask (or None).
    """

    @staticmethod
    def forward(ctx, cfg: FrontendCfg, wave, dummy, gn_w, gn_b, *wm):
        layers = cfg.layers
        n = len(layers)
        ws_ = list(wm[0::2])
        masks = list(wm[1::2])
        B, S = wave.shape
        Ls = conv_lengths(S, layers)
        dev = wave.device
        need = cfg.need_grad
        C0, k0, s0 = layers[0]
        C0p = pad8(C0)
        # conv0 of a pruned student (ragged C0) runs over C0p channels with zero weights / affine /
        # mask in the padding: those channels come out exactly 0
        w0, g0, b0, m0 = ws_[0], gn_w, gn_b, masks[0]
        if C0p != C0:
            w0 = torch.zeros(C0p, *ws_[0].shape[1:], dtype=F32, device=dev)
            w0[:C0] = ws_[0].detach()
            g0, b0 = padded_vec(gn_w.detach(), C0p), padded_vec(gn_b.detach(), C0p)
            m0 = padded_vec(masks[0] if masks[0] is not None else torch.ones(C0, device=dev), C0p)
        y = torch.empty(B * Ls[0], C0p, dtype=BF16, device=dev)
        mean = torch.empty(B, C0p, dtype=F32, device=dev)
        rstd = torch.empty(B, C0p, dtype=F32, device=dev)
        ws = torch.empty(B * 16 * 65 * 2, dtype=F32, device=dev)   # per-(utterance, chunk) fp64 Gram partials
        call("dph_conv0_gn_fwd", ptr(wave), B, S, ptr(w0), C0p, k0, s0, ptr(g0), ptr(b0), ptr(m0),
             ptr(y), ptr(mean), ptr(rstd), ptr(ws), ws.numel() * 4, _s())
        ys, zs, imgs, cms = [y], [None], [None], [m0]
        Cin, Cinp = C0, C0p
        for i in range(1, n):
            O, k, s = layers[i]
            Op = pad8(O)
            img = conv_image(ws_[i], Op, Cinp)
            cm = masks[i]
            if i == n - 1:
                cm = dummy if cm is None else cm * dummy
            cm = padded_vec(cm, Op)
            out = torch.empty(B * Ls[i], Op, dtype=BF16, device=dev)
            z = torch.empty(B * Ls[i], Op, dtype=BF16, device=dev) if need else None
            A = K.mat(ys[-1], row_stride=s * Cinp, rows_per_batch=Ls[i], batch_stride=Ls[i - 1] * Cinp)
            K.gemm(A, K.dense(img), K.dense(out), B * Ls[i], Op, k * Cinp, a_kcontig=True, b_kcontig=True,
                   act=K.ACT_GELU, pre_out=z, colmask=cm)
            ys.append(out)
            zs.append(z)
            imgs.append(img)
            cms.append(cm)
            Cin, Cinp = O, Op
        if need:
            ctx.cfg = cfg
            ctx.params = (gn_w, gn_b, *ws_)
            ctx.Ls = Ls
            ctx.cms = cms
            ctx.has_mask = [m is not None for m in masks]
            ctx.padded0 = (w0, g0, b0, m0) if C0p != C0 else None
            ctx.save_for_backward(wave, dummy, gn_w, gn_b, mean, rstd, *ws_, *[m if m is not None else dummy
                                                                            for m in masks])
            ctx.ys = ys[:-1]   # inputs of layers 1..n-1 (the last output is not needed)
            ctx.zs = zs
            ctx.imgs = imgs
        return ys[-1]

    @staticmethod
    def backward(ctx, dy):
        cfg = ctx.cfg
        layers = cfg.layers
        n = len(layers)
        saved = ctx.saved_tensors
        wave, dummy, gn_w, gn_b, mean, rstd = saved[:6]
        ws_ = list(saved[6:6 + n])
        masks = [m if h else None for m, h in zip(saved[6 + n:6 + 2 * n], ctx.has_mask)]
        Ls = ctx.Ls
        B, S = wave.shape
        dev = wave.device
        dy = dy.contiguous()
        pgn_w, pgn_b, *pws = ctx.params
        go = GradOut(dev)
        g_m = [None] * n
        # last layer: GELU / (mask*dummy) backward (widths are the 8-padded storage widths)
        O = layers[-1][0]
        Op = pad8(O)
        dz = torch.empty_like(dy)
        dm_raw = zeros_f32(Op, dev)
        call("dph_gelu_mask_bwd", ptr(dy), ptr(ctx.zs[-1]), ptr(ctx.cms[-1]), ptr(dz), ptr(dm_raw), B * Ls[-1], Op,
             *rb_ws(B * Ls[-1], Op, dev), _s())
        if masks[-1] is not None:
            g_m[-1] = dm_raw[:O] * dummy
        keep = []
        for i in range(n - 1, 0, -1):
            O, k, s = layers[i]
            Op = pad8(O)
            Cin = layers[i - 1][0]
            Cinp = pad8(Cin)
            M = B * Ls[i]
            # weight gradient (packed [O][k*Cinp]) -> [O][Cin][k]
            dw, direct = go.buf(pws[i], zero=False)
            with wgrad_side(dz, ctx.ys[i - 1], enable=direct, scope="conv"):
                dwp = torch.empty(O, k * Cinp, dtype=F32, device=dev)
                A = K.mat(dz, row_stride=Op)
                Bm = K.mat(ctx.ys[i - 1], row_stride=s * Cinp, rows_per_batch=Ls[i], batch_stride=Ls[i - 1] * Cinp)
                splits = K.choose_splits(O, k * Cinp, M)
                keep.append(K.gemm(A, Bm, K.dense(dwp), O, k * Cinp, M, a_kcontig=False, b_kcontig=False,
                                   c_dtype=K.OUT_F32, splits=splits, device=dev))
                call("dph_conv_weight_unpack_grad", ptr(dwp), ptr(dw), O, Cin, k, Cinp, int(direct), _s())
                keep.append(dwp)
            # input gradient, fused with the previous layer's GELU/mask backward (i > 1): phase GEMMs
            # writing d_in in place, or the column gradient + col2im for other conv geometries
            wt = t_image(ctx.imgs[i])     # [k*Cinp][Op]: both operands k-contiguous -> ring kernels
            dmk = (zeros_f32(Cinp, dev) if masks[i - 1] is not None else zeros_f32(Cinp, dev)) if i > 1 else None
            nxt = None
            if wt is not None and _PHASE_DGRAD:
                nxt = conv_dgrad_phases(dz, wt, B, Ls[i], Ls[i - 1], Op, Cinp, k, s,
                                        z_pre=ctx.zs[i - 1] if i > 1 else None,
                                        cm=ctx.cms[i - 1] if i > 1 else None, dmask=dmk)
            if nxt is None:
                dcols = torch.empty(M, k * Cinp, dtype=BF16, device=dev)
                if wt is not None:
                    K.gemm(K.dense(dz), K.dense(wt), K.dense(dcols), M, k * Cinp, Op, a_kcontig=True, b_kcontig=True)
                else:
                    K.gemm(K.dense(dz), K.dense(ctx.imgs[i]), K.dense(dcols), M, k * Cinp, Op, a_kcontig=True,
                           b_kcontig=False)
                nxt = torch.empty(B * Ls[i - 1], Cinp, dtype=BF16, device=dev)
                if i > 1:
                    call("dph_col2im_gelu_bwd", ptr(dcols), B, Ls[i], Ls[i - 1], Cinp, k, s, ptr(ctx.zs[i - 1]),
                         ptr(ctx.cms[i - 1]), ptr(nxt), ptr(dmk), *rb_ws(B * Ls[i - 1], Cinp, dev), _s())
                else:
                    call("dph_col2im_gelu_bwd", ptr(dcols), B, Ls[i], Ls[i - 1], Cinp, k, s, None, None, ptr(nxt),
                         None, None, 0, _s())
            if i > 1 and masks[i - 1] is not None:
                g_m[i - 1] = dmk[:Cin]
            dz = nxt
        # layer 0: conv0 + GroupNorm + GELU + mask, recomputed from the waveform
        C0, k0, s0 = layers[0]
        C0p = pad8(C0)
        if ctx.padded0 is None:
            dw0, _ = go.buf(pws[0])
            dgw, _ = go.buf(pgn_w)
            dgb, _ = go.buf(pgn_b)
            w0, g0, b0, m0 = ws_[0], gn_w, gn_b, masks[0]
        else:   # pruned (ragged) conv0: padded scratch gradients, returned sliced to autograd
            w0, g0, b0, m0 = ctx.padded0
            dw0, dgw, dgb = zeros_f32((C0p,) + tuple(ws_[0].shape[1:]), dev), zeros_f32(C0p, dev), zeros_f32(C0p, dev)
            go.bufs[id(pws[0])], go.bufs[id(pgn_w)], go.bufs[id(pgn_b)] = dw0[:C0], dgw[:C0], dgb[:C0]
        dm0 = zeros_f32(C0p, dev) if masks[0] is not None else None
        wsb = torch.empty((_lib.lib().dph_conv0_gn_bwd_workspace(B, S, C0p) + 3) // 4, dtype=F32, device=dev)
        call("dph_conv0_gn_bwd", ptr(wave), B, S, ptr(w0), C0p, k0, s0, ptr(g0), ptr(b0), ptr(m0),
             ptr(mean), ptr(rstd), ptr(dz), ptr(dw0), ptr(dgw), ptr(dgb), ptr(dm0), ptr(wsb), wsb.numel() * 4, _s())
        g_m[0] = dm0[:C0] if dm0 is not None else None
        go.done()
        grads = [None, None, None, go.ret(pgn_w), go.ret(pgn_b)]
        for i in range(n):
            grads += [go.ret(pws[i]), g_m[i]]
        return tuple(grads)


# ---------------------------------------------------------------------------
# Feature projection: LN(C) -> Linear(C->D) -> dropout -> zero padded frames
# ---------------------------------------------------------------------------
class FrontendLNFn(torch.autograd.Function):
    """layer_norm-mode FeatureExtractor (HuBERT-Large / wav2vec2-Large-LV60 teachers;
    components.py:54-61 LayerNorm wrapper, :107-120 ConvLayerBlock, :137-185): every layer is
    conv (+bias) -> LayerNorm over channels -> exact GELU -> x HardConcrete channel mask, the
    last output times dummy_weight.  conv0 is the register-window FIR (dph_conv0_fwd), conv1-6 the
    implicit GEMMs with the bias in the epilogue; LayerNorm, GELU*mask and their backward are the
    dense kernels; conv0's weight / bias gradients come from dph_conv0_bwd.

    inputs: wave, dummy_weight, then per layer: conv weight, conv bias (or None), LN weight, LN
    bias, mask (or None).  Channel counts must be multiples of 8 (no ragged pruned students here).
    """

    @staticmethod
    def forward(ctx, cfg: FrontendCfg, wave, dummy, *pl):
        layers = cfg.layers
        n = len(layers)
        ps = [pl[5 * i:5 * i + 5] for i in range(n)]
        for (C, _, _) in layers:
            if C % 8:
                raise NotImplementedError("layer_norm-mode extractor with a ragged (pruned) conv width")
        B, S = wave.shape
        Ls = conv_lengths(S, layers)
        dev = wave.device
        need = cfg.need_grad
        zs, hs, ys, stats, cms, imgs = [], [], [], [], [], []
        C0, k0, s0 = layers[0]
        for i in range(n):
            w, bias, lw, lb, m = ps[i]
            C, k, s = layers[i]
            rows = B * Ls[i]
            # pre-LN conv outputs in fp32 (conv0's FIR output is bf16): seven bf16-rounded pre-LN
            # tensors put the hidden states 1.02e-2 rel-L2 from the fp32 reference (> the 1e-2 bar)
            if i == 0:
                z = torch.empty(rows, C, dtype=BF16, device=dev)
                call("dph_conv0_fwd", ptr(wave), B, S, ptr(w), ptr(bias), C, k, s, ptr(z), _s())
                imgs.append(None)
            else:
                z = torch.empty(rows, C, dtype=F32, device=dev)
                Cin = layers[i - 1][0]
                img = conv_image(w, C, Cin)
                A = K.mat(ys[-1], row_stride=s * Cin, rows_per_batch=Ls[i], batch_stride=Ls[i - 1] * Cin)
                K.gemm(A, K.dense(img), K.dense(z), rows, C, k * Cin, a_kcontig=True, b_kcontig=True, bias=bias,
                       c_dtype=K.OUT_F32)
                imgs.append(img)
            h = torch.empty(rows, C, dtype=BF16, device=dev) if need else None
            mu = torch.empty(rows, dtype=F32, device=dev)
            rs = torch.empty(rows, dtype=F32, device=dev)
            cm = m
            if i == n - 1:
                cm = dummy if cm is None else cm * dummy
            y = torch.empty(rows, C, dtype=BF16, device=dev)
            # LN + GELU + mask in one pass (GELU of the fp32 LN value); h = bf16 LN output for backward
            call("dph_layernorm_gelu_fwd", ptr(z), int(z.dtype == F32), ptr(lw), ptr(lb), ptr(h), ptr(cm), ptr(y),
                 ptr(mu), ptr(rs), rows, C, 1e-5, _s())
            zs.append(z)
            hs.append(h)
            ys.append(y)
            stats.append((mu, rs))
            cms.append(cm)
        if need:
            ctx.cfg = cfg
            ctx.params = pl
            ctx.Ls = Ls
            ctx.has_mask = [p[4] is not None for p in ps]
            ctx.has_bias = [p[1] is not None for p in ps]
            ctx.zs, ctx.hs, ctx.ys, ctx.stats, ctx.cms, ctx.imgs = zs, hs, ys[:-1], stats, cms, imgs
            ctx.save_for_backward(wave, dummy)
        return ys[-1]

    @staticmethod
    def backward(ctx, dy):
        cfg = ctx.cfg
        layers = cfg.layers
        n = len(layers)
        wave, dummy = ctx.saved_tensors
        ps = [ctx.params[5 * i:5 * i + 5] for i in range(n)]
        Ls = ctx.Ls
        B, S = wave.shape
        dev = wave.device
        go = GradOut(dev)
        g_m = [None] * n
        C = layers[-1][0]
        rows = B * Ls[-1]
        dh = torch.empty(rows, C, dtype=BF16, device=dev)
        dm = zeros_f32(C, dev)
        call("dph_gelu_mask_bwd", ptr(dy.contiguous()), ptr(ctx.hs[-1]), ptr(ctx.cms[-1]), ptr(dh), ptr(dm), rows, C,
             *rb_ws(rows, C, dev), _s())
        if ctx.has_mask[-1]:
            g_m[-1] = dm * dummy
        keep = []
        for i in range(n - 1, -1, -1):
            w, bias, lw, lb, m = ps[i]
            C, k, s = layers[i]
            rows = B * Ls[i]
            mu, rs = ctx.stats[i]
            dz = torch.empty(rows, C, dtype=BF16, device=dev)
            dlw, _ = go.buf(lw)
            dlb, _ = go.buf(lb)
            if ctx.zs[i].dtype == F32:
                call("dph_layernorm_bwd_x32", ptr(dh), ptr(ctx.zs[i]), ptr(lw), ptr(mu), ptr(rs), ptr(dz), ptr(dlw),
                     ptr(dlb), rows, C, *ln_ws(rows, C, dev), _s())
            else:
                call("dph_layernorm_bwd", ptr(dh), ptr(ctx.zs[i]), None, ptr(lw), ptr(mu), ptr(rs), ptr(dz),
                     ptr(dlw), ptr(dlb), rows, C, 0.0, 0, None, 0.0, 0, None, None, None, None,
                     *ln_ws(rows, C, dev), _s())
            if bias is not None:
                dbias, _ = go.buf(bias)
                call("dph_colsum", ptr(dz), ptr(dbias), rows, C, *colsum_ws(rows, C, dev), _s())
            if i == 0:
                dw, direct = go.buf(w)
                call("dph_conv0_bwd", ptr(wave), B, S, C, k, s, ptr(dz), ptr(dw), None,
                     *_ws(_lib.lib().dph_conv0_bwd_workspace(B, S, C), dev), _s())
                break
            Cin = layers[i - 1][0]
            dwp = torch.empty(C, k * Cin, dtype=F32, device=dev)
            A = K.mat(dz, row_stride=C)
            Bm = K.mat(ctx.ys[i - 1], row_stride=s * Cin, rows_per_batch=Ls[i], batch_stride=Ls[i - 1] * Cin)
            splits = K.choose_splits(C, k * Cin, rows)
            keep.append(K.gemm(A, Bm, K.dense(dwp), C, k * Cin, rows, a_kcontig=False, b_kcontig=False,
                               c_dtype=K.OUT_F32, splits=splits, device=dev))
            dw, direct = go.buf(w, zero=False)
            call("dph_conv_weight_unpack_grad", ptr(dwp), ptr(dw), C, Cin, k, Cin, int(direct), _s())
            wt = t_image(ctx.imgs[i])
            dmk = zeros_f32(Cin, dev)
            dh = None
            if wt is not None and _PHASE_DGRAD:
                dh = conv_dgrad_phases(dz, wt, B, Ls[i], Ls[i - 1], C, Cin, k, s, z_pre=ctx.hs[i - 1],
                                       cm=ctx.cms[i - 1], dmask=dmk)
            if dh is None:
                dcols = torch.empty(rows, k * Cin, dtype=BF16, device=dev)
                if wt is not None:
                    K.gemm(K.dense(dz), K.dense(wt), K.dense(dcols), rows, k * Cin, C, a_kcontig=True, b_kcontig=True)
                else:
                    K.gemm(K.dense(dz), K.dense(ctx.imgs[i]), K.dense(dcols), rows, k * Cin, C, a_kcontig=True,
                           b_kcontig=False)
                dh = torch.empty(B * Ls[i - 1], Cin, dtype=BF16, device=dev)
                call("dph_col2im_gelu_bwd", ptr(dcols), B, Ls[i], Ls[i - 1], Cin, k, s, ptr(ctx.hs[i - 1]),
                     ptr(ctx.cms[i - 1]), ptr(dh), ptr(dmk), *rb_ws(B * Ls[i - 1], Cin, dev), _s())
            if ctx.has_mask[i - 1]:
                g_m[i - 1] = dmk
        # the conv0 weight gradient went through dph_conv0_bwd, which accumulates (needs a zeroed
        # buffer when it is not the bucket itself: GradOut.buf zero-fills by default)
        go.done()
        grads = [None, None, None]
        for i, (w, bias, lw, lb, m) in enumerate(ps):
            grads += [go.ret(w), go.ret(bias) if bias is not None else None, go.ret(lw), go.ret(lb), g_m[i]]
        return tuple(grads)


class FeatureProjectionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ln_w, ln_b, w, b, cfg):
        # x: [M][Cp] with the true channel count C = cfg["C"] <= Cp (8-padded rows of a pruned
        # frontend; the padding columns are zero and stay zero through LN)
        M, Cp = x.shape
        C = cfg.get("C") or Cp
        dev = x.device
        xn = torch.empty_like(x)
        mu = torch.empty(M, dtype=F32, device=dev)
        rs = torch.empty(M, dtype=F32, device=dev)
        call("dph_layernorm_fwd_ld", ptr(x), None, ptr(ln_w), ptr(ln_b), ptr(xn), ptr(mu), ptr(rs), M, C, Cp, 1e-5,
             0.0, 0, _s())
        img = padded_image(w, w.shape[0], Cp)
        seed = SEEDS.next() if cfg["p"] > 0 else 0
        out = K.linear_fwd(xn, img, b, dropout_p=cfg["p"], seed=seed, row_len=cfg["lengths"],
                           len_rows=cfg["T"] if cfg["lengths"] is not None else 0)
        ctx.cfg = cfg
        ctx.seed = seed
        ctx.params = (ln_w, ln_b, w, b)
        ctx.save_for_backward(x, xn, mu, rs, ln_w, img)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, xn, mu, rs, ln_w, img = ctx.saved_tensors
        cfg = ctx.cfg
        M, Cp = x.shape
        C = cfg.get("C") or Cp
        D = img.shape[0]
        dev = x.device
        dout = dout.contiguous()
        dpre = torch.empty_like(dout)
        p_lw, p_lb, p_w, p_b = ctx.params
        go = GradOut(dev)
        db, _ = go.buf(p_b)
        lens = cfg["lengths"]
        call("dph_branch_bwd", ptr(dout), ptr(dpre), M, D, cfg["p"], ctx.seed, None, ptr(lens),
             cfg["T"] if lens is not None else 0, ptr(db), None, None, *rb_ws(M, D, dev), _s())
        dw, direct = go.buf(p_w, zero=False)
        ws = K.linear_wgrad(dpre, xn, dw, accumulate=direct, k_in=C)
        dxn = K.linear_dgrad(dpre, img, w_t=t_image(img))
        dx = torch.empty_like(x)
        dlw, _ = go.buf(p_lw)
        dlb, _ = go.buf(p_lb)
        call("dph_layernorm_bwd_ld", ptr(dxn), ptr(x), None, ptr(ln_w), ptr(mu), ptr(rs), ptr(dx), ptr(dlw), ptr(dlb),
             M, C, Cp, 0.0, 0, None, 0.0, 0, None, None, None, None, None, *ln_ws(M, C, dev), _s())
        del ws
        go.done()
        return dx, go.ret(p_lw), go.ret(p_lb), go.ret(p_w), go.ret(p_b), None


# ---------------------------------------------------------------------------
# Positional conv embedding + residual + LayerNorm + dropout (Transformer._preprocess)
# ---------------------------------------------------------------------------
def _weight_norm_ws(R: int, K: int, dev):
    """Workspace of the deterministic per-tap reduction in dph_weight_norm_{fwd,bwd} (64 rows/block)."""
    return torch.empty(-(-R // 64) * K, dtype=F32, device=dev)


class LayerNormFn(torch.autograd.Function):
    """Plain nn.LayerNorm over the last dim of (rows, D) (the final LN of a pre-norm Transformer.forward,
    components.py:903-904): x bf16, or fp32 -- the pre-norm layers' fp32 residual stream -- with a bf16 output."""

    @staticmethod
    def forward(ctx, x, w, b):
        M, D = x.shape
        y = torch.empty(M, D, dtype=BF16, device=x.device)
        mu = torch.empty(M, dtype=F32, device=x.device)
        rs = torch.empty(M, dtype=F32, device=x.device)
        if x.dtype == F32:
            call("dph_layernorm_fwd_x32", ptr(x), ptr(w), ptr(b), ptr(y), ptr(mu), ptr(rs), M, D, 1e-5, _s())
        else:
            call("dph_layernorm_fwd", ptr(x), None, ptr(w), ptr(b), ptr(y), ptr(mu), ptr(rs), M, D, 1e-5, 0.0, 0, _s())
        ctx.save_for_backward(x, w, mu, rs)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, mu, rs = ctx.saved_tensors
        M, D = x.shape
        dy = dy.contiguous()
        if dy.dtype != BF16:
            dy = dy.to(BF16)
        dx = torch.empty_like(x)
        dw = zeros_f32(D, x.device)
        db = zeros_f32(D, x.device)
        if x.dtype == F32:
            call("dph_layernorm_bwd_res32", ptr(dy), ptr(x), ptr(w), ptr(mu), ptr(rs), ptr(dx), ptr(dw), ptr(db), M, D,
                 None, *ln_ws(M, D, x.device), _s())
        else:
            call("dph_layernorm_bwd", ptr(dy), ptr(x), None, ptr(w), ptr(mu), ptr(rs), ptr(dx), ptr(dw), ptr(db), M, D,
                 0.0, 0, None, 0.0, 0, None, None, None, None, *ln_ws(M, D, x.device), _s())
        return dx, dw, db


def invalidate_weight_norm_cache(module: torch.nn.Module) -> int:
    """Drop the cached positional-conv weight-norm images of a frozen module (PosConvFn): needed after writing its
    weights in a way that does not bump their version counters (``.data`` writes).  Returns how many were dropped.
    Captured HIP graphs that replayed a cached image must be recaptured too (Trainer._drop_graphs)."""
    n = 0
    for p in module.parameters():
        if getattr(p, "_dph_wn_img", None) is not None:
            p._dph_wn_img = None
            n += 1
    return n


class PosConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wg, wv, bias, ln_w, ln_b, cfg):
        B, T, G = cfg["B"], cfg["T"], cfg["G"]
        M, D = x.shape
        Kk = wv.shape[2]
        Cg = D // G
        dev = x.device
        # weight norm -> bf16 GEMM images (forward and flipped/transposed for dgrad).  A frozen model's (the
        # teacher's: no gradient, parameters without requires_grad) forward image is computed once per weight
        # version and reused: the step graph then carries no weight-norm launches for it.  ASSUMPTION: a frozen
        # weight changes only through ops that bump its version (load_state_dict, copy_, the DDP broadcast); an
        # in-place write through .data or an alias with its own version counter does not -- call
        # invalidate_weight_norm_cache(module) after one.  A graph captured after a cache hit replays the cached
        # image (it does not re-read wg / wv).
        frozen = not cfg["need_grad"] and not wg.requires_grad and not wv.requires_grad
        key = (wg.data_ptr(), wg._version, wv.data_ptr(), wv._version, G, Kk)
        hit = getattr(wv, "_dph_wn_img", None) if frozen else None
        if hit is not None and hit[0] == key:
            norm, wk, wt = hit[1], hit[2], None
        else:
            norm = torch.empty(Kk, dtype=F32, device=dev)
            wk = torch.empty(G, Cg, Kk * Cg, dtype=BF16, device=dev)
            wt = None if frozen else torch.empty(G, Cg, Kk * Cg, dtype=BF16, device=dev)
            wn_ws = _weight_norm_ws(D * Cg, Kk, dev)
            call("dph_weight_norm_fwd", ptr(wg), ptr(wv), D, Cg, Kk, G, None, ptr(norm), ptr(wk), ptr(wt),
                 ptr(wn_ws), wn_ws.numel() * 4, _s())
            if frozen and not torch.cuda.is_current_stream_capturing():
                wv._dph_wn_img = (key, norm, wk)
        P = Kk // 2
        Q = Kk - 1 - P
        Tp = P + T + Q
        xg = torch.empty(B * G * Tp * Cg, dtype=BF16, device=dev)
        call("dph_regroup_pad", ptr(x), ptr(xg), B, T, G, Cg, P, Q, _s())
        need = cfg["need_grad"]
        ln = cfg.get("ln", True)
        # pre-norm Transformer: s0 = x + pos_conv(x) starts the fp32 residual stream of the layers (EncoderLayerFn)
        s0 = torch.empty_like(x) if ln else torch.empty(M, D, dtype=F32, device=dev)
        z = torch.empty_like(x) if need else None
        Cm = K.mat(s0, D, z_div=G, z_outer=T * D, z_inner=Cg)
        K.gemm(K.mat(xg, Cg, z_inner=Tp * Cg), K.mat(wk, Kk * Cg, z_div=G, z_outer=0, z_inner=Cg * Kk * Cg), Cm, T,
               Cg, Kk * Cg, a_kcontig=True, b_kcontig=True, batch=B * G, act=K.ACT_GELU, bias=bias, vec_z_inner=Cg,
               pre_out=z, residual=x, c_dtype=K.OUT_BF16 if ln else K.OUT_F32)
        mu = torch.empty(M, dtype=F32, device=dev)
        rs = torch.empty(M, dtype=F32, device=dev)
        seed = SEEDS.next() if cfg["p"] > 0 else 0
        if ln:
            h = torch.empty_like(x)
            call("dph_layernorm_fwd", ptr(s0), None, ptr(ln_w), ptr(ln_b), ptr(h), ptr(mu), ptr(rs), M, D, 1e-5,
                 cfg["p"], seed, _s())
        elif cfg["p"] > 0:   # pre-norm Transformer (components.py:1283 flag): no LayerNorm here, dropout only
            h = torch.empty(M, D, dtype=F32, device=dev)
            call("dph_branch_bwd_f32", ptr(s0), ptr(h), 1, M, D, cfg["p"], seed, None, None, 0, None, None, None,
                 None, 0, _s())
        else:
            h = s0
        if need:
            ctx.cfg = cfg
            ctx.seed = seed
            ctx.params = (bias, ln_w, ln_b)
            ctx.save_for_backward(x, wg, wv, norm, wt, xg, s0, z, mu, rs, ln_w)
        return h

    @staticmethod
    def backward(ctx, dh):
        x, wg, wv, norm, wt, xg, s0, z, mu, rs, ln_w = ctx.saved_tensors
        cfg = ctx.cfg
        B, T, G = cfg["B"], cfg["T"], cfg["G"]
        M, D = x.shape
        Kk = wv.shape[2]
        Cg = D // G
        dev = x.device
        dh = dh.contiguous()
        ds0 = torch.empty(M, D, dtype=BF16, device=dev)
        p_bias, p_lw, p_lb = ctx.params
        go = GradOut(dev)
        if cfg.get("ln", True):
            dlw, _ = go.buf(p_lw)
            dlb, _ = go.buf(p_lb)
            call("dph_layernorm_bwd", ptr(dh), ptr(s0), None, ptr(ln_w), ptr(mu), ptr(rs), ptr(ds0), ptr(dlw),
                 ptr(dlb), M, D, cfg["p"], ctx.seed, None, 0.0, 0, None, None, None, None, *ln_ws(M, D, dev), _s())
        else:   # (the fp32 residual stream's gradient)
            dh = dh if dh.dtype == F32 else dh.float()
            call("dph_branch_bwd_f32", ptr(dh), ptr(ds0), 0, M, D, cfg["p"], ctx.seed, None, None, 0, None, None,
                 None, None, 0, _s())
        # (+64 elements of slack: the weight gradient below reads 64 columns from group g's first one, see there)
        dz = torch.empty(M * D + 64, dtype=BF16, device=dev)[:M * D].view(M, D)
        call("dph_gelu_mask_bwd", ptr(ds0), ptr(z), None, ptr(dz), None, M, D, None, 0, _s())
        db, _ = go.buf(p_bias)
        call("dph_colsum", ptr(dz), ptr(db), M, D, *colsum_ws(M, D, dev), _s())
        # input gradient: transposed conv = same batched GEMM over a re-padded dz with flipped weights
        P = Kk // 2
        Q = Kk - 1 - P
        P2, Q2 = Kk - 1 - P, Kk - 1 - Q
        Tp2 = P2 + T + Q2
        dzg = torch.empty(B * G * Tp2 * Cg, dtype=BF16, device=dev)
        call("dph_regroup_pad", ptr(dz), ptr(dzg), B, T, G, Cg, P2, Q2, _s())
        dx = torch.empty_like(x)
        K.gemm(K.mat(dzg, Cg, z_inner=Tp2 * Cg), K.mat(wt, Kk * Cg, z_div=G, z_outer=0, z_inner=Cg * Kk * Cg),
               K.mat(dx, D, z_div=G, z_outer=T * D, z_inner=Cg), T, Cg, Kk * Cg, a_kcontig=True, b_kcontig=True,
               batch=B * G, residual=ds0)
        # weight gradient in GEMM image layout [G][Cg_out][K*Cg_in].  The ping-pong (mn, mn) kernel takes M >= 64:
        # a group's Cg = 48 output channels run as Mp = 64 GEMM rows (the 16 extra read the next group's dz columns
        # -- or the slack past the last row -- and land in rows that are dropped); DPH_POSCONV_MP=0 keeps M = Cg on the
        # register-staged kernel (A/B)
        Tp = P + T + Q
        Mp = 64 if (Cg < 64 and Cg % 8 == 0 and os.environ.get("DPH_POSCONV_MP", "1") != "0") else Cg
        dimg_p = torch.empty(G, Mp, Kk * Cg, dtype=F32, device=dev)
        A = K.mat(dz, D, z_inner=Cg)
        Bm = K.mat(xg, Cg, rows_per_batch=T, batch_stride=G * Tp * Cg, z_inner=Tp * Cg)
        splits = K.choose_splits(Mp, Kk * Cg, B * T, batch=G)
        ws = K.gemm(A, Bm, K.mat(dimg_p, Kk * Cg, z_inner=Mp * Kk * Cg), Mp, Kk * Cg, B * T, a_kcontig=False,
                    b_kcontig=False, c_dtype=K.OUT_F32, batch=G, splits=splits, device=dev)
        dimg = dimg_p[:, :Cg].contiguous() if Mp != Cg else dimg_p
        dg = torch.empty_like(norm)
        dv = torch.empty_like(wv)
        wn_ws = _weight_norm_ws(D * Cg, Kk, dev)
        call("dph_weight_norm_bwd", ptr(dimg), ptr(wg), ptr(wv), ptr(norm), D, Cg, Kk, G, ptr(dg), ptr(dv), ptr(wn_ws),
             wn_ws.numel() * 4, _s())
        del ws
        go.done()
        return dx, dg.view_as(wg), dv, go.ret(p_bias), go.ret(p_lw), go.ret(p_lb), None


# ---------------------------------------------------------------------------
# Encoder layer (post-norm; HuBERT/wav2vec2 Base)
# ---------------------------------------------------------------------------
class RelPosTableFn(torch.autograd.Function):
    """WavLM position bias (compute_bias, components.py:546-561) as one value per diagonal:
    embed [num_buckets][H] fp32 -> rel_tab [H][2T-1] fp32, rel_tab[h][r] = embed[bucket(r-(T-1))][h].
    Backward scatters the diagonal gradients back into the embedding rows (Embedding backward)."""

    @staticmethod
    def forward(ctx, embed, T, num_buckets, max_distance):
        if not embed.is_cuda:
            raise ValueError("RelPosTableFn: the HIP path needs device tensors")
        Htot = embed.shape[1]
        e = embed.detach().contiguous()
        tab = torch.empty(Htot, 2 * T - 1, dtype=F32, device=embed.device)
        call("dph_relpos_table", ptr(e), None, ptr(tab), None, T, Htot, Htot, num_buckets, max_distance, _s())
        ctx.meta = (embed, T, num_buckets, max_distance)
        return tab

    @staticmethod
    def backward(ctx, dtab):
        embed, T, nb, md = ctx.meta
        go = GradOut(embed.device)
        de, _ = go.buf(embed)
        call("dph_relpos_table_bwd", ptr(dtab.contiguous()), None, ptr(de), T, embed.shape[1], embed.shape[1], nb, md,
             _s())
        go.done()
        return go.ret(embed), None, None, None


def _ffn_dgk(D: int) -> bool:
    """The FFN intermediate GELU backward from factors the forward stores (K.GEMM_PRE_DGK / K.ACT_GELU_BWD_DGK):
    the forward GEMM keeps gelu'(pre)*mask*keep/(1-p) instead of pre, so the input-gradient GEMM's epilogue is
    two multiplies (no erfc, no dropout hash; the mask gradient from the stored output f / mask).  Needs the
    ping-pong GEMM layout (K = D a multiple of 64, >= 128) for both operands k-contiguous -- so the transposed
    weight images too (DPH_DGRAD_T=0 turns them off, and with them this path); DPH_FFN_DGK=0 keeps the recomputing
    epilogue (A/B)."""
    return _DGRAD_T and D % 64 == 0 and D >= 128 and os.environ.get("DPH_FFN_DGK", "1") != "0"


def _ffn_interm_bwd(dy, sv, db1, dmask, cfg, F_):
    """du = (dy @ W2) * gelu'(pre) * mask * keep/(1-p); db1 += colsum(du); dmask += colsum((dy @ W2) * gelu(pre) *
    keep/(1-p)) (components.py:733-739 backward)."""
    if sv["dgk"]:
        # dmask None: the mask gradient comes from the FFN2 weight gradient (dph_colprod), f is not read here
        return K.linear_dgrad(dy, sv["W2"], w_t=t_image(sv["W2"]), act=K.ACT_GELU_BWD_DGK, aux_in=sv["u"],
                              residual=sv["f"] if dmask is not None else None, colmask=sv["imp"], colsum_out=db1,
                              colsum_aux=dmask, colsum_n=F_)
    return K.linear_dgrad(dy, sv["W2"], w_t=t_image(sv["W2"]), act=K.ACT_GELU_BWD, aux_in=sv["u"], colmask=sv["imp"],
                          colsum_out=db1, colsum_aux=dmask, dropout_p=cfg["p_interm"], seed=sv["seed_i"], colsum_n=F_)



@K.tagged("ffn")
def _ffn_forward(cfg, xin, w1, b1, w2, b2, im, lmf, resid, need, sv):
    """FeedForward (components.py:726-748) + dropout + layer mask + residual: resid + drop(FFN(xin)) * lmf.

    Training with sampled intermediate masks (``im``, HardConcrete interm units): the units whose mask is exactly
    0 (hardconcrete.py:99 clamps) are dropped from every FFN GEMM -- dph_ffn_compact packs the active ones to the
    front of Fc-wide images (W1 rows, W2 columns, b1, mask) and the GEMMs read the active extent from device
    memory (DphGemmArgs.dyn_ext), so the captured step graph keeps fixed shapes.  The FFN1 dropout then hashes the
    packed column index (the same keep rate, another draw than the full-width layout would take).
    Taken where cfg["ffn_compact"] is set (the trainer's choice from the gate's expected zero fraction: the
    packing / unpacking launches cost ~10 us per layer, measured to pay off from ~30 % zero units); DPH_FFN_COMPACT=1 / 0
    forces it on / off (tests, A/B)."""
    M, D = xin.shape
    dev = xin.device
    # intermediate width F of a pruned student is ragged: stored 8-padded (zero weight rows /
    # columns, bias and mask padding 0 -> the padding columns of u and f are exactly 0)
    F_ = w1.shape[0]
    Fp = pad8(F_)
    W1 = padded_image(w1, Fp, D)
    W2 = padded_image(w2, D, Fp)
    b1p, imp = padded_vec(b1, Fp), padded_vec(im, Fp)
    seed_i = SEEDS.next() if cfg["p_interm"] > 0 else 0
    dgk = _ffn_dgk(D) and need
    seed_o = SEEDS.next() if cfg["p_drop"] > 0 else 0
    y_pre = torch.empty(M, D, dtype=BF16, device=dev) if (need and lmf is not None) else None
    mode = os.environ.get("DPH_FFN_COMPACT", "auto")
    compact = mode == "1" or (mode != "0" and cfg.get("ffn_compact", False))
    if dgk and im is not None and compact and Fp <= 8192:
        Fc = max(128, (Fp + 63) // 64 * 64)
        idx = torch.empty(Fc, dtype=torch.int32, device=dev)
        ext = torch.empty(10, dtype=torch.int32, device=dev)
        call("dph_ffn_compact", ptr(imp), Fp, Fc, ptr(idx), ptr(ext), _s())
        # every packed operand of the forward AND the backward GEMMs in one launch (W1 rows, W2 columns, the rows /
        # columns of their transposed images, b1, mask)
        W1t, W2t = t_image(W1), t_image(W2)
        W1g = torch.empty(Fc, D, dtype=BF16, device=dev)
        W2g = torch.empty(D, Fc, dtype=BF16, device=dev)
        W2gT = torch.empty(Fc, D, dtype=BF16, device=dev) if W2t is not None else None
        W1gT = torch.empty(D, Fc, dtype=BF16, device=dev) if W1t is not None else None
        b1g = torch.empty(Fc, dtype=F32, device=dev)
        mg = torch.empty(Fc, dtype=F32, device=dev)
        call("dph_ffn_pack", ptr(W1), ptr(W2), ptr(W2t), ptr(W1t), ptr(b1p), ptr(imp), ptr(idx), ptr(W1g), ptr(W2g),
             ptr(W2gT), ptr(W1gT), ptr(b1g), ptr(mg), Fp, Fc, D, _s())
        u = torch.empty(M, Fc, dtype=BF16, device=dev)
        f = K.linear_fwd(xin, W1g, b1g, act=K.ACT_GELU, pre_out=u, colmask=mg, dropout_p=cfg["p_interm"],
                         seed=seed_i, pre_dgk=True, dyn=(ext, 0))
        out = K.linear_fwd(f, W2g, b2, smask=lmf, residual=resid, dropout_p=cfg["p_drop"], seed=seed_o,
                           pre_out=y_pre, dyn=(ext, 3))
        sv.update(W1=W1, W2=W2, W1g=W1g, W2g=W2g, W1gT=W1gT, W2gT=W2gT, idx=idx, ext=ext, Fc=Fc, u=u, f=f,
                  y_pre=y_pre, seed_i=seed_i, seed_o=seed_o, F=F_, imp=mg, dgk=True, compact=True)
        return out
    u = torch.empty(M, Fp, dtype=BF16, device=dev) if need else None
    f = K.linear_fwd(xin, W1, b1p, act=K.ACT_GELU, pre_out=u, colmask=imp, dropout_p=cfg["p_interm"],
                     seed=seed_i, pre_dgk=dgk)
    out = K.linear_fwd(f, W2, b2, smask=lmf, residual=resid, dropout_p=cfg["p_drop"], seed=seed_o, pre_out=y_pre)
    sv.update(W1=W1, W2=W2, u=u, f=f, y_pre=y_pre, seed_i=seed_i, seed_o=seed_o, F=F_, imp=imp, dgk=dgk,
              compact=False)
    return out


@K.tagged("ffn")
def _ffn_backward(cfg, sv, dy, xin, pr, go, dmask, residual=None):
    """Backward of _ffn_forward from dy = d(FFN2 output) (after the output dropout / layer mask): the W2 / b1 / W1
    gradients into ``go``'s buffers, the intermediate-mask gradient into ``dmask`` [F] (None: no intermediate mask,
    not computed), returns d(xin) (+ residual)."""
    M, D = xin.shape
    dev = xin.device
    F_ = sv["F"]
    if sv["compact"]:
        Fc, idx, ext = sv["Fc"], sv["idx"], sv["ext"]
        dW2g = torch.empty(D, Fc, dtype=F32, device=dev)
        k1 = K.linear_wgrad(dy, sv["f"], dW2g, accumulate=False, dyn=(ext, 0))
        db1g, dmg = zeros_f32(Fc, dev), zeros_f32(Fc, dev)
        W2gT = sv["W2gT"] if sv["W2gT"] is not None else sv["W2g"].t().contiguous()
        du = K.linear_dgrad(dy, sv["W2g"], w_t=W2gT, act=K.ACT_GELU_BWD_DGK, aux_in=sv["u"], residual=sv["f"],
                            colmask=sv["imp"], colsum_out=db1g, colsum_aux=dmg, colsum_n=Fc, dyn=(ext, 0))
        dW1g = torch.empty(Fc, D, dtype=F32, device=dev)
        k2 = K.linear_wgrad(du, xin, dW1g, accumulate=False, dyn=(ext, 6))
        W1gT = sv["W1gT"] if sv["W1gT"] is not None else sv["W1g"].t().contiguous()
        dx = K.linear_dgrad(du, sv["W1g"], w_t=W1gT, residual=residual, dyn=(ext, 3))
        # the packed gradients back to the full-width (bucket) ones in one launch (accumulating: the buffers are the
        # zeroed-at-step-start buckets or zero-filled)
        dw2, _ = go.buf(pr["w2"], zero=True)
        dw1, _ = go.buf(pr["w1"], zero=True)
        db1, _ = go.buf(pr["b1"])
        call("dph_ffn_unpack_grads", ptr(dW2g), ptr(dW1g), ptr(db1g), ptr(dmg), ptr(idx), ptr(dw2), F_, ptr(dw1),
             ptr(db1), ptr(dmask), Fc, D, _s())
        del k1, k2
        return dx
    dw2, direct = go.buf(pr["w2"], zero=False)
    # the mask gradient as sum_o W2[o][n] dW2[o][n] / mask_n over THIS micro-batch's dW2 = dY^T f: a fresh buffer,
    # or a bucket zeroed at this micro-batch's start (gradient accumulation past the first micro-batch, and the
    # weight-gradient side stream, keep the f-reading epilogue)
    colprod = (_FFN_COLPROD and sv["dgk"] and dmask is not None and _WGRAD_SIDE[0] is None
               and ((not direct) or _bucket_fresh(pr["w2"])))
    post = None
    if colprod:
        W2i, imp = sv["W2"], sv["imp"]
        post = lambda: call("dph_colprod", ptr(W2i), W2i.shape[1], ptr(dw2), F_, ptr(imp), ptr(dmask), D, F_,  # noqa
                            _s())
    k1 = _layer_wgrad(dy, sv["f"], dw2, direct, (pr["w2"],), post=post, k_in=F_)
    db1, db1d = go.buf(pr["b1"])
    dmk = None if colprod else dmask
    with _defer_red(go, db1d, dmk is None):     # (the mask gradient feeds autograd: never queued)
        du = _ffn_interm_bwd(dy, sv, db1, dmk, cfg, F_)
    dw1, direct = go.buf(pr["w1"], zero=False)
    k2 = _layer_wgrad(du, xin, dw1, direct, (pr["w1"],), n_out=F_)
    dx = K.linear_dgrad(du, sv["W1"], w_t=t_image(sv["W1"]), residual=residual)
    del k1, k2
    return dx


class EncoderLayerFn(torch.autograd.Function):
    """h (B*T, D) bf16 -> layer output (B*T, D) bf16.

    tensors: h, wq, wk, wv, bq, bk, bv, wo, bo, ln1_w, ln1_b, w1, b1, w2, b2, ln2_w, ln2_b,
             head_mask, att_lmask, interm_mask, ff_lmask   (masks may be None; attention /
             FFN weights may be None when the sub-layer is pruned away)
    """

    @staticmethod
    def forward(ctx, cfg, h, wq, wk, wv, bq, bk, bv, wo, bo, ln1_w, ln1_b, w1, b1, w2, b2, ln2_w, ln2_b, hm, lma,
                im, lmf, rel_tab=None, gw=None, gb=None, gc=None, heads=None):
        ctx.wl = dict(rel_tab=rel_tab, gw=gw, gb=gb, gc=gc, heads=heads) if rel_tab is not None else None
        if cfg.get("pre_norm"):
            return EncoderLayerFn._forward_pre(ctx, cfg, h, wq, wk, wv, bq, bk, bv, wo, bo, ln1_w, ln1_b, w1, b1, w2,
                                               b2, ln2_w, ln2_b, hm, lma, im, lmf)
        ctx.pre = False
        M, D = h.shape
        dev = h.device
        need = cfg["need_grad"]
        B, T, H = cfg["B"], cfg["T"], cfg["H"]
        use_att = wq is not None
        use_ff = w1 is not None
        sv = {}
        # ---------------- attention block ----------------
        if use_att:
            Dh = wq.shape[0]
            Wqkv = bf16_image(wq, wk, wv)
            bqkv = f32_cat(bq, bk, bv)
            qkv = K.linear_fwd(h, Wqkv, bqkv)
            # fp32 unmasked output: the backward's D (attention.hip); neither it nor the LSE is written without a
            # backward (the teacher)
            o_u = torch.empty(M, Dh, dtype=F32, device=dev) if (need or _TEACHER_OU) else None
            o_m = torch.empty(M, Dh, dtype=BF16, device=dev)
            lse = torch.empty(B * H * T, dtype=F32, device=dev) if (need or _TEACHER_OU) else None
            seed_a = SEEDS.next() if cfg["p_attn"] > 0 else 0
            sv["gate"] = EncoderLayerFn._attention_fwd(ctx, cfg, h, qkv, o_u, o_m, lse, hm, seed_a)
            Wo = bf16_image(wo)
            seed_d = SEEDS.next() if cfg["p_drop"] > 0 else 0
            a_pre = torch.empty(M, D, dtype=BF16, device=dev) if (need and lma is not None) else None
            s1 = K.linear_fwd(o_m, Wo, bo, smask=lma, residual=h, dropout_p=cfg["p_drop"], seed=seed_d,
                              pre_out=a_pre)
            sv.update(Wqkv=Wqkv, qkv=qkv, o_u=o_u, o_m=o_m, lse=lse, Wo=Wo, a_pre=a_pre, seed_a=seed_a, seed_d=seed_d)
        else:
            s1 = h
        h1 = torch.empty_like(h)
        mu1 = torch.empty(M, dtype=F32, device=dev)
        rs1 = torch.empty(M, dtype=F32, device=dev)
        call("dph_layernorm_fwd", ptr(s1), None, ptr(ln1_w), ptr(ln1_b), ptr(h1), ptr(mu1), ptr(rs1), M, D, 1e-5, 0.0,
             0, _s())
        # ---------------- feed-forward block ----------------
        if use_ff:
            s2 = _ffn_forward(cfg, h1, w1, b1, w2, b2, im, lmf, h1, need, sv)
        else:
            s2 = h1
        out = torch.empty_like(h)
        mu2 = torch.empty(M, dtype=F32, device=dev)
        rs2 = torch.empty(M, dtype=F32, device=dev)
        call("dph_layernorm_fwd", ptr(s2), None, ptr(ln2_w), ptr(ln2_b), ptr(out), ptr(mu2), ptr(rs2), M, D, 1e-5,
             0.0, 0, _s())
        if need:
            ctx.cfg = cfg
            ctx.sv = sv
            ctx.params = dict(wq=wq, wk=wk, wv=wv, bq=bq, bk=bk, bv=bv, wo=wo, bo=bo, ln1_w=ln1_w, ln1_b=ln1_b, w1=w1,
                              b1=b1, w2=w2, b2=b2, ln2_w=ln2_w, ln2_b=ln2_b)
            ctx.flags = (use_att, use_ff, hm is not None, lma is not None, im is not None, lmf is not None)
            ctx.save_for_backward(h, s1, mu1, rs1, h1, s2, mu2, rs2, ln1_w, ln2_w, hm, lma, im, lmf)
        return out

    # ---------------- pre-norm (wav2vec2 / HuBERT Large, components.py:835-845) ----------------
    #   s1  = h + drop(attn(LN1(h))) * layer_mask_att
    #   out = s1 + FFN(LN2(s1)) * layer_mask_ffn        (no LayerNorm after the block)
    # The residual stream h -> s1 -> out is fp32 (and so is its gradient): a bf16 stream takes two roundings per
    # layer of an un-normalised sum (48 over wav2vec2-Large's 24 layers) -- the GEMM epilogues add the branch to the
    # fp32 residual (DPH_GEMM_RESID_F32), the LayerNorms read it in fp32 and write the bf16 GEMM operand.
    @staticmethod
    def _forward_pre(ctx, cfg, h, wq, wk, wv, bq, bk, bv, wo, bo, ln1_w, ln1_b, w1, b1, w2, b2, ln2_w, ln2_b, hm,
                     lma, im, lmf):
        if h.dtype != F32:
            raise ValueError("pre-norm encoder layers carry the residual stream in fp32 (got %s)" % h.dtype)
        M, D = h.shape
        dev = h.device
        need = cfg["need_grad"]
        B, T, H = cfg["B"], cfg["T"], cfg["H"]
        use_att = wq is not None
        use_ff = w1 is not None
        sv = {}
        xn1 = mu1 = rs1 = xn2 = mu2 = rs2 = None
        if use_att:
            xn1 = torch.empty(M, D, dtype=BF16, device=dev)
            mu1 = torch.empty(M, dtype=F32, device=dev)
            rs1 = torch.empty(M, dtype=F32, device=dev)
            call("dph_layernorm_fwd_x32", ptr(h), ptr(ln1_w), ptr(ln1_b), ptr(xn1), ptr(mu1), ptr(rs1), M, D, 1e-5,
                 _s())
            Dh = wq.shape[0]
            Wqkv = bf16_image(wq, wk, wv)
            qkv = K.linear_fwd(xn1, Wqkv, f32_cat(bq, bk, bv))
            o_u = torch.empty(M, Dh, dtype=F32, device=dev) if need else None   # (as the post-norm forward)
            o_m = torch.empty(M, Dh, dtype=BF16, device=dev)
            lse = torch.empty(B * H * T, dtype=F32, device=dev) if need else None
            seed_a = SEEDS.next() if cfg["p_attn"] > 0 else 0
            sv["gate"] = EncoderLayerFn._attention_fwd(ctx, cfg, xn1, qkv, o_u, o_m, lse, hm, seed_a)
            Wo = bf16_image(wo)
            seed_d = SEEDS.next() if cfg["p_drop"] > 0 else 0
            a_pre = torch.empty(M, D, dtype=BF16, device=dev) if (need and lma is not None) else None
            s1 = K.linear_fwd(o_m, Wo, bo, smask=lma, residual=h, dropout_p=cfg["p_drop"], seed=seed_d,
                              pre_out=a_pre)                  # fp32 (fp32 residual)
            sv.update(Wqkv=Wqkv, qkv=qkv, o_u=o_u, o_m=o_m, lse=lse, Wo=Wo, a_pre=a_pre, seed_a=seed_a, seed_d=seed_d)
        else:
            s1 = h
        if use_ff:
            xn2 = torch.empty(M, D, dtype=BF16, device=dev)
            mu2 = torch.empty(M, dtype=F32, device=dev)
            rs2 = torch.empty(M, dtype=F32, device=dev)
            call("dph_layernorm_fwd_x32", ptr(s1), ptr(ln2_w), ptr(ln2_b), ptr(xn2), ptr(mu2), ptr(rs2), M, D, 1e-5,
                 _s())
            out = _ffn_forward(cfg, xn2, w1, b1, w2, b2, im, lmf, s1, need, sv)
        else:
            out = s1.clone() if s1 is h else s1
        if need:
            ctx.pre = True
            ctx.cfg = cfg
            ctx.sv = sv
            ctx.params = dict(wq=wq, wk=wk, wv=wv, bq=bq, bk=bk, bv=bv, wo=wo, bo=bo, ln1_w=ln1_w, ln1_b=ln1_b, w1=w1,
                              b1=b1, w2=w2, b2=b2, ln2_w=ln2_w, ln2_b=ln2_b)
            ctx.flags = (use_att, use_ff, hm is not None, lma is not None, im is not None, lmf is not None)
            ctx.save_for_backward(h, xn1, mu1, rs1, s1, xn2, mu2, rs2, ln1_w, ln2_w, hm, lma, im, lmf)
        return out

    @staticmethod
    def _backward_pre(ctx, dout):
        h, xn1, mu1, rs1, s1, xn2, mu2, rs2, ln1_w, ln2_w, hm, lma, im, lmf = ctx.saved_tensors
        cfg = ctx.cfg
        sv = ctx.sv
        use_att, use_ff, has_hm, has_lma, has_im, has_lmf = ctx.flags
        B, T, H = cfg["B"], cfg["T"], cfg["H"]
        M, D = h.shape
        dev = h.device
        dout = dout.contiguous()
        if dout.dtype != F32:
            dout = dout.float()
        z = lambda n: zeros_f32(n, dev)  # noqa: E731
        pr = ctx.params
        go = GradOut(dev)
        g = {}
        # ---- FFN branch: out = s1 + drop(FFN(LN2(s1))) * lmf  (dout, ds1: fp32 residual-stream gradients) ----
        if use_ff:
            dy = torch.empty(M, D, dtype=BF16, device=dev)
            db2, _ = go.buf(pr["b2"])
            g["lmf"] = z(1) if has_lmf else None
            call("dph_branch_bwd_f32", ptr(dout), ptr(dy), 0, M, D, cfg["p_drop"], sv["seed_o"], ptr(lmf), None, 0,
                 ptr(db2), ptr(sv["y_pre"]) if has_lmf else None, ptr(g["lmf"]), *rb_ws(M, D, dev), _s())
            F_ = sv["F"]
            g["im"] = z(F_) if has_im else None
            dxn2 = _ffn_backward(cfg, sv, dy, xn2, pr, go, g["im"])
            ds1 = torch.empty(M, D, dtype=F32, device=dev)
            dln2w, _ = go.buf(pr["ln2_w"])
            dln2b, _ = go.buf(pr["ln2_b"])
            call("dph_layernorm_bwd_res32", ptr(dxn2), ptr(s1), ptr(ln2_w), ptr(mu2), ptr(rs2), ptr(ds1), ptr(dln2w),
                 ptr(dln2b), M, D, ptr(dout), *ln_ws(M, D, dev), _s())
        else:
            ds1 = dout
        # ---- attention branch: s1 = h + drop(attn(LN1(h))) * lma ----
        if use_att:
            da = torch.empty(M, D, dtype=BF16, device=dev)
            dbo, _ = go.buf(pr["bo"])
            g["lma"] = z(1) if has_lma else None
            call("dph_branch_bwd_f32", ptr(ds1), ptr(da), 0, M, D, cfg["p_drop"], sv["seed_d"], ptr(lma), None, 0,
                 ptr(dbo), ptr(sv["a_pre"]) if has_lma else None, ptr(g["lma"]), *rb_ws(M, D, dev), _s())
            dwo, direct = go.buf(pr["wo"], zero=False)
            k3 = _layer_wgrad(da, sv["o_m"], dwo, direct, (pr["wo"],))
            do_m = K.linear_dgrad(da, sv["Wo"], w_t=t_image(sv["Wo"]))
            Dvec = torch.empty(B * H * T, dtype=F32, device=dev)
            g["hm"] = z(H) if has_hm else None
            call("dph_attention_bwd_prep", ptr(do_m), ptr(sv["o_u"]), ptr(hm), ptr(Dvec), ptr(g["hm"]), B, T, H,
                 *_ws(_lib.lib().dph_attention_bwd_prep_workspace(B, T, H), dev), _s())
            dqkv = torch.empty_like(sv["qkv"])
            dbqkv, _ = go.buf(pr["bq"], pr["bk"], pr["bv"])
            wl_g = EncoderLayerFn._attention_bwd(ctx, cfg, sv, do_m, hm, Dvec, dqkv, dbqkv)
            dwqkv, direct = go.buf(pr["wq"], pr["wk"], pr["wv"], zero=False)
            k4 = _layer_wgrad(dqkv, xn1, dwqkv, direct, (pr["wq"], pr["wk"], pr["wv"]))
            dxn1 = K.linear_dgrad(dqkv, sv["Wqkv"], w_t=t_image(sv["Wqkv"]))
            EncoderLayerFn._gate_bwd(ctx, cfg, xn1, dxn1, wl_g, go)
            dh = torch.empty(M, D, dtype=F32, device=dev)
            dln1w, _ = go.buf(pr["ln1_w"])
            dln1b, _ = go.buf(pr["ln1_b"])
            call("dph_layernorm_bwd_res32", ptr(dxn1), ptr(h), ptr(ln1_w), ptr(mu1), ptr(rs1), ptr(dh), ptr(dln1w),
                 ptr(dln1b), M, D, ptr(ds1), *ln_ws(M, D, dev), _s())
            del k3, k4
        else:
            dh = ds1
        go.done()
        order = ["wq", "wk", "wv", "bq", "bk", "bv", "wo", "bo", "ln1_w", "ln1_b", "w1", "b1", "w2", "b2", "ln2_w",
                 "ln2_b"]
        return (None, dh) + tuple(go.ret(pr[k]) for k in order) + (g.get("hm"), g.get("lma"), g.get("im"),
                                                                    g.get("lmf")) + EncoderLayerFn._wl_ret(ctx, go)

    # ---------------- WavLM gated relative-position bias (components.py:629-651) ----------------
    @staticmethod
    def _attention_fwd(ctx, cfg, x_att, qkv, o_u, o_m, lse, hm, seed_a):
        """Attention forward; with a WavLM bias the per-query gate is computed from the attention input first
        (dph_wavlm_gate_fwd) and the kernels add gate * rel_tab[k-q] to the scores.  Returns the gate."""
        B, T, H = cfg["B"], cfg["T"], cfg["H"]
        wl = ctx.wl
        # attention dropout: the forward stores its keep bits (1 bit per probability, ~6 MB per layer at B=16) and
        # the backward kernels read them instead of re-hashing every probability twice (grad mode is off inside an
        # autograd.Function forward, so the caller's need_grad decides)
        keep = None
        if cfg["p_attn"] > 0 and cfg.get("need_grad", True):
            keep = torch.empty(_lib.lib().dph_attention_keep_bytes(B, T, H) // 8, dtype=torch.int64, device=qkv.device)
        ctx.attn_keep = keep
        if wl is None:
            call("dph_attention_fwd", ptr(qkv), ptr(o_u), ptr(o_m), ptr(lse), ptr(hm), ptr(cfg["lengths"]), B, T, H,
                 cfg["head_dim"] ** -0.5, cfg["p_attn"], seed_a, ptr(keep), _s())
            return None
        if cfg["head_dim"] != 64:
            raise NotImplementedError("WavLM gate: head_dim 64 only")
        gate = torch.empty(B * H * T, dtype=F32, device=qkv.device)
        call("dph_wavlm_gate_fwd", ptr(x_att), x_att.shape[1], ptr(wl["gw"]), ptr(wl["gb"]), ptr(wl["gc"]),
             ptr(wl["heads"]), ptr(gate), B, T, H, 64, _s())
        wl["rel_tab"] = wl["rel_tab"].contiguous()
        call("dph_attention_fwd_relpos", ptr(qkv), ptr(o_u), ptr(o_m), ptr(lse), ptr(hm), ptr(cfg["lengths"]),
             ptr(wl["rel_tab"]), ptr(gate), B, T, H, cfg["head_dim"] ** -0.5, cfg["p_attn"], seed_a, ptr(keep), _s())
        return gate

    @staticmethod
    def _attention_bwd(ctx, cfg, sv, do_m, hm, Dvec, dqkv, dbqkv):
        """dq | dk | dv into dqkv, and the q / v bias gradients added into dbqkv's [bq | bk | bv] (summed inside the
        backward kernels: dph_attention_bwd_qv; DPH_KBIAS_GRAD=1 -- the k bias as well -- or DPH_ATTN_QV=0 takes the
        plain backward and the separate column sums of dqkv)."""
        B, T, H = cfg["B"], cfg["T"], cfg["H"]
        wl = ctx.wl
        dev = dqkv.device
        M = B * T
        fused = _ATTN_QV and not _KBIAS_GRAD
        L = _lib.lib()
        # one scratch tensor, held until the call, for the relpos slab (WavLM, deterministic mode) and the q / v bias
        # slab (a released _ws block would be handed out again to the dgate / dtab allocations below)
        rws = L.dph_attention_bwd_relpos_workspace(B, T, H) if wl is not None else 0
        rws = (rws + 255) // 256 * 256
        qvb = L.dph_attention_bwd_qv_workspace(B, T, H) if fused else 0
        wst = _ws_t(rws + qvb, dev)
        wsp = ptr(wst)
        if fused:
            Dh = dqkv.shape[1] // 3
            base = dbqkv.data_ptr()
            qv = (base, base + 8 * Dh, wsp + rws, qvb)
        if wl is None:
            args = (ptr(sv["qkv"]), ptr(do_m), ptr(hm), ptr(sv["lse"]), ptr(Dvec), ptr(dqkv), ptr(cfg["lengths"]), B, T,
                    H, cfg["head_dim"] ** -0.5, cfg["p_attn"], sv["seed_a"], ptr(getattr(ctx, "attn_keep", None)))
            if fused:
                call("dph_attention_bwd_qv", *args, *qv, _s())
            else:
                call("dph_attention_bwd", *args, _s())
                _qkv_bias_grad(dqkv, dbqkv, M, dev)
            return None
        dgate = torch.empty(B * H * T, dtype=F32, device=dev)
        dtab = torch.zeros(wl["rel_tab"].shape, dtype=F32, device=dev)
        args = (ptr(sv["qkv"]), ptr(do_m), ptr(hm), ptr(sv["lse"]), ptr(Dvec), ptr(dqkv), ptr(cfg["lengths"]),
                ptr(wl["rel_tab"]), ptr(sv["gate"]), ptr(dgate), ptr(dtab), B, T, H, cfg["head_dim"] ** -0.5,
                cfg["p_attn"], sv["seed_a"], ptr(getattr(ctx, "attn_keep", None)), wsp, rws)
        if fused:
            call("dph_attention_bwd_relpos_qv", *args, *qv, _s())
        else:
            call("dph_attention_bwd_relpos", *args, _s())
            _qkv_bias_grad(dqkv, dbqkv, M, dev)
        del wst
        return dgate, dtab

    @staticmethod
    def _gate_bwd(ctx, cfg, x_att, dx_att, wl_g, go):
        """The gate's backward: its input gradient is added into dx_att (the attention input's gradient)."""
        wl = ctx.wl
        if wl is None:
            return
        B, T, H = cfg["B"], cfg["T"], cfg["H"]
        dgate, dtab = wl_g
        dgw, _ = go.buf(wl["gw"])
        dgb, _ = go.buf(wl["gb"])
        dgc, _ = go.buf(wl["gc"])
        N = B * T * H
        ws = torch.empty(_lib.lib().dph_wavlm_gate_bwd_workspace(B, T, H) // 4, dtype=F32, device=dx_att.device)
        call("dph_wavlm_gate_bwd", ptr(x_att), x_att.shape[1], ptr(wl["gw"]), ptr(wl["gb"]), ptr(wl["gc"]),
             ptr(wl["heads"]), ptr(dgate), ptr(dx_att), dx_att.shape[1], ptr(dgw), ptr(dgb), ptr(dgc), ptr(ws),
             ws.numel() * 4, B, T, H, 64, _s())
        wl["dtab"] = dtab

    @staticmethod
    def _wl_ret(ctx, go):
        wl = ctx.wl
        if wl is None:
            return (None,) * 5
        return (wl.get("dtab"), go.ret(wl["gw"]), go.ret(wl["gb"]), go.ret(wl["gc"]), None)

    @staticmethod
    def backward(ctx, dout):
        if ctx.pre:
            return EncoderLayerFn._backward_pre(ctx, dout)
        h, s1, mu1, rs1, h1, s2, mu2, rs2, ln1_w, ln2_w, hm, lma, im, lmf = ctx.saved_tensors
        cfg = ctx.cfg
        sv = ctx.sv
        use_att, use_ff, has_hm, has_lma, has_im, has_lmf = ctx.flags
        B, T, H = cfg["B"], cfg["T"], cfg["H"]
        M, D = h.shape
        dev = h.device
        dout = dout.contiguous()
        z = lambda n: zeros_f32(n, dev)  # noqa: E731
        pr = ctx.params
        go = GradOut(dev)
        g = {}
        # ---- LN2 backward (+ FFN branch gradient) ----
        ds2 = torch.empty_like(dout)
        dln2w, d2w = go.buf(pr["ln2_w"])
        dln2b, d2b = go.buf(pr["ln2_b"])
        if use_ff:
            dy = torch.empty_like(dout)
            db2, dd2 = go.buf(pr["b2"])
            g["lmf"] = z(1) if has_lmf else None
            with _defer_red(go, d2w, d2b, dd2):
                call("dph_layernorm_bwd", ptr(dout), ptr(s2), None, ptr(ln2_w), ptr(mu2), ptr(rs2), ptr(ds2),
                     ptr(dln2w), ptr(dln2b), M, D, 0.0, 0, ptr(dy), cfg["p_drop"], sv["seed_o"], ptr(lmf), ptr(db2),
                     ptr(sv["y_pre"]), ptr(g["lmf"]), *ln_ws(M, D, dev), _s())
            F_ = sv["F"]
            g["im"] = z(F_) if has_im else None
            dh1 = _ffn_backward(cfg, sv, dy, h1, pr, go, g["im"], residual=ds2)
        else:
            with _defer_red(go, d2w, d2b):
                call("dph_layernorm_bwd", ptr(dout), ptr(s2), None, ptr(ln2_w), ptr(mu2), ptr(rs2), ptr(ds2),
                     ptr(dln2w), ptr(dln2b), M, D, 0.0, 0, None, 0.0, 0, None, None, None, None, *ln_ws(M, D, dev),
                     _s())
            dh1 = ds2
        # ---- LN1 backward (+ attention branch gradient) ----
        ds1 = torch.empty_like(dout)
        dln1w, d1w = go.buf(pr["ln1_w"])
        dln1b, d1b = go.buf(pr["ln1_b"])
        if use_att:
            da = torch.empty_like(dout)
            dbo, ddo = go.buf(pr["bo"])
            g["lma"] = z(1) if has_lma else None
            with _defer_red(go, d1w, d1b, ddo):
                call("dph_layernorm_bwd", ptr(dh1), ptr(s1), None, ptr(ln1_w), ptr(mu1), ptr(rs1), ptr(ds1),
                     ptr(dln1w), ptr(dln1b), M, D, 0.0, 0, ptr(da), cfg["p_drop"], sv["seed_d"], ptr(lma), ptr(dbo),
                     ptr(sv["a_pre"]), ptr(g["lma"]), *ln_ws(M, D, dev), _s())
            dwo, direct = go.buf(pr["wo"], zero=False)
            k3 = _layer_wgrad(da, sv["o_m"], dwo, direct, (pr["wo"],))
            do_m = K.linear_dgrad(da, sv["Wo"], w_t=t_image(sv["Wo"]))
            Dvec = torch.empty(B * H * T, dtype=F32, device=dev)
            g["hm"] = z(H) if has_hm else None
            call("dph_attention_bwd_prep", ptr(do_m), ptr(sv["o_u"]), ptr(hm), ptr(Dvec), ptr(g["hm"]), B, T, H,
                 *_ws(_lib.lib().dph_attention_bwd_prep_workspace(B, T, H), dev), _s())
            dqkv = torch.empty_like(sv["qkv"])
            dbqkv, dqb = go.buf(pr["bq"], pr["bk"], pr["bv"])
            with _defer_red(go, dqb):
                wl_g = EncoderLayerFn._attention_bwd(ctx, cfg, sv, do_m, hm, Dvec, dqkv, dbqkv)
            dwqkv, direct = go.buf(pr["wq"], pr["wk"], pr["wv"], zero=False)
            k4 = _layer_wgrad(dqkv, h, dwqkv, direct, (pr["wq"], pr["wk"], pr["wv"]))
            dh = K.linear_dgrad(dqkv, sv["Wqkv"], w_t=t_image(sv["Wqkv"]), residual=ds1)
            EncoderLayerFn._gate_bwd(ctx, cfg, h, dh, wl_g, go)
            del k3, k4
        else:
            with _defer_red(go, d1w, d1b):
                call("dph_layernorm_bwd", ptr(dh1), ptr(s1), None, ptr(ln1_w), ptr(mu1), ptr(rs1), ptr(ds1),
                     ptr(dln1w), ptr(dln1b), M, D, 0.0, 0, None, 0.0, 0, None, None, None, None, *ln_ws(M, D, dev),
                     _s())
            dh = ds1
        go.done()
        order = ["wq", "wk", "wv", "bq", "bk", "bv", "wo", "bo", "ln1_w", "ln1_b", "w1", "b1", "w2", "b2", "ln2_w",
                 "ln2_b"]
        return (None, dh) + tuple(go.ret(pr[k]) for k in order) + (g.get("hm"), g.get("lma"), g.get("im"),
                                                                    g.get("lmf")) + EncoderLayerFn._wl_ret(ctx, go)


# ---------------------------------------------------------------------------
# Distill projections + DistillLoss (fused)
# ---------------------------------------------------------------------------
def _bf16_rows(xs):
    """bf16 copies of the fp32 tensors of ``xs`` (one per distinct tensor; bf16 ones pass through)."""
    done = {}
    out = []
    for x in xs:
        if x.dtype == BF16:
            out.append(x)
            continue
        if id(x) not in done:
            y = torch.empty(x.shape, dtype=BF16, device=x.device)
            call("dph_cast_bf16", ptr(x.contiguous()), ptr(y), x.numel(), _s())
            done[id(x)] = y
        out.append(done[id(x)])
    return out


class DistillProjLossFn(torch.autograd.Function):
    """student hidden list -> per-layer Linear (shared per group) -> loss terms.

    args: cfg, then L student hiddens (B*T, Ds) bf16, then P projection (weight, bias) pairs,
    then L teacher hiddens (B*T, Dt) bf16.  Returns (loss, mse, l1, cos) 0-d fp32.
    Hiddens of pre-norm encoders are the fp32 residual stream (EncoderLayerFn._forward_pre): the student's are
    rounded to bf16 once here (the projection GEMM's operand) and their gradients are fp32; the loss kernel reads
    the teacher's in fp32.
    """

    @staticmethod
    def forward(ctx, cfg, *args):
        L, P = cfg["L"], cfg["P"]
        sh = args[:L]
        pw = args[L:L + 2 * P]
        th = args[L + 2 * P:L + 2 * P + L]
        B, T = cfg["B"], cfg["T"]
        M, Ds = sh[0].shape
        Dt = pw[0].shape[0]
        dev = sh[0].device
        ctx.in_f32 = [x.dtype == F32 for x in sh]
        sh = _bf16_rows(sh)          # (the projection GEMM's operand; the teacher rows are read in their dtype)
        tmask = sum(1 << l for l, t in enumerate(th) if t.dtype == F32)
        ctx.tmask = tmask
        s = torch.empty(L, M, Dt, dtype=F32, device=dev)
        imgs = [bf16_image(pw[2 * p]) for p in range(P)]
        # predlayer heads (distill.py:100-107): Linear + exact-erf GELU in the GEMM epilogue, the pre-activation
        # kept in bf16 for the backward
        gelu = cfg.get("head_act") == "gelu"
        pre = torch.empty(L, M, Dt, dtype=BF16, device=dev) if gelu else None
        for l in range(L):
            p = cfg["proj_index"][l]
            if gelu:
                K.linear_fwd(sh[l], imgs[p], pw[2 * p + 1], out=s[l], act=K.ACT_GELU, pre_out=pre[l])
            else:
                K.linear_fwd(sh[l], imgs[p], pw[2 * p + 1], out=s[l])
        rowstats = torch.empty(L * M * 3, dtype=F32, device=dev)
        partial = torch.empty(LOSS_PARTIAL_FLOATS, dtype=F32, device=dev)
        out = torch.empty(4, dtype=F32, device=dev)
        tptrs = (_lib.C.c_void_p * L)(*[t.data_ptr() for t in th])
        call("dph_distill_loss_fwd_ex", ptr(s), tptrs, tmask, B, L, T, Dt, cfg["l2"], cfg["l1"], cfg["cos"],
             int(cfg["cos_type"] == "log_sig"), ptr(rowstats), ptr(partial), ptr(out), _s())
        ctx.cfg = cfg
        ctx.params = pw
        ctx.pre = pre
        ctx.save_for_backward(s, rowstats, *sh, *imgs, *th)
        return out[0], out[1], out[2], out[3]

    @staticmethod
    def backward(ctx, dloss, dmse, dl1, dcos):
        cfg = ctx.cfg
        L, P = cfg["L"], cfg["P"]
        s, rowstats, *rest = ctx.saved_tensors
        sh = rest[:L]
        imgs = rest[L:L + P]
        th = rest[L + P:]
        B, T = cfg["B"], cfg["T"]
        M, Ds = sh[0].shape
        Dt = s.shape[2]
        dev = s.device
        ds = torch.empty(L, M, Dt, dtype=BF16, device=dev)
        tptrs = (_lib.C.c_void_p * L)(*[t.data_ptr() for t in th])
        dl = dloss.contiguous() if dloss is not None else torch.ones((), dtype=F32, device=dev)
        call("dph_distill_loss_bwd_ex", ptr(s), tptrs, ctx.tmask, ptr(rowstats), ptr(dl), B, L, T, Dt, cfg["l2"],
             cfg["l1"], cfg["cos"], int(cfg["cos_type"] == "log_sig"), ptr(ds), _s())
        go = GradOut(dev)
        pw = ctx.params
        dW = [go.buf(pw[2 * p])[0] for p in range(P)]
        dbs = [go.buf(pw[2 * p + 1]) for p in range(P)]
        db = [t for t, _ in dbs]
        db_direct = [d for _, d in dbs]
        if ctx.pre is not None:
            # through the heads' GELU: dz = ds * gelu'(pre), in place
            call("dph_gelu_mask_bwd", ptr(ds), ptr(ctx.pre), None, ptr(ds), None, L * M, Dt, None, 0, _s())
            ctx.pre = None
        # predlayer: every head reads the same (last) hidden state -> one chained input gradient
        shared = cfg.get("shared_input", False)
        dh = []
        keep = []
        acc = None
        for l in range(L):
            p = cfg["proj_index"][l]
            keep.append(K.linear_wgrad(ds[l], sh[l], dW[p], accumulate=True))
            with _defer_red(go, db_direct[p]):
                call("dph_colsum", ptr(ds[l]), ptr(db[p]), M, Dt, *colsum_ws(M, Dt, dev), _s())
            o = torch.empty(M, Ds, dtype=F32, device=dev) if ctx.in_f32[l] else None
            if shared:
                acc = K.linear_dgrad(ds[l], imgs[p], w_t=t_image(imgs[p]), residual=acc, out=o if acc is None else None)
            else:
                dh.append(K.linear_dgrad(ds[l], imgs[p], w_t=t_image(imgs[p]), out=o))
        if shared:
            dh = [acc] + [None] * (L - 1)
        go.done()
        grads = [None] + dh
        for p in range(P):
            grads += [go.ret(pw[2 * p]), go.ret(pw[2 * p + 1])]
        grads += [None] * L
        return tuple(grads)
