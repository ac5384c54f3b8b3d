"""Thin tensor-level wrappers over the C ABI (one function per entry point).

Each wrapper validates shapes/dtypes/devices on the host, then passes raw
device pointers and the current HIP stream to libdphubert_hip.so.  Scratch
buffers are allocated here through the PyTorch caching allocator, never
inside the library.
"""

import ctypes as C
import os
from typing import Optional, Sequence

import torch

from . import _lib
from ._lib import DphGemmArgs, DphMat, call, ptr

BF16 = torch.bfloat16
F32 = torch.float32
_SPLITK_INLAUNCH = __import__("os").environ.get("DPH_SPLITK_INLAUNCH", "0") == "1"

ACT_NONE, ACT_GELU, ACT_GELU_BWD, ACT_GELU_BWD_DGK = 0, 1, 2, 3
OUT_BF16, OUT_F32, OUT_F32_ACCUM = 0, 1, 2


def _stream():
    return _lib.stream_ptr()


def _chk(t, dtype=None, name="tensor"):
    if t is None:
        return
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor (no CPU path)")
    if dtype is not None and t.dtype != dtype:
        raise ValueError(f"{name}: expected {dtype}, got {t.dtype}")


def mat(t: torch.Tensor, row_stride: int, rows_per_batch: int = 0, batch_stride: int = 0, z_div: int = 0,
        z_outer: int = 0, z_inner: int = 0, offset: int = 0) -> DphMat:
    """Describe a strided 2-D (optionally batched) view of ``t`` for the GEMM."""
    return DphMat(t.data_ptr() + offset * t.element_size(), rows_per_batch, batch_stride, row_stride, z_div, z_outer,
                  z_inner)


def dense(t: torch.Tensor, offset: int = 0, row_stride: Optional[int] = None) -> DphMat:
    return mat(t, t.shape[-1] if row_stride is None else row_stride, offset=offset)


class _Event:
    """A hipEvent_t from the kernel library: recorded as an external event node when the launch
    stream is being captured (torch refuses external events on ROCm)."""

    def __init__(self):
        h = C.c_void_p()
        call("dph_event_create", C.byref(h))
        self.h = h.value

    def record(self):
        call("dph_event_record", self.h, _stream())

    def elapsed_time(self, end: "_Event") -> float:
        ms = C.c_float()
        call("dph_event_elapsed_ms", self.h, end.h, C.byref(ms))
        return ms.value

    def __del__(self):
        try:
            _lib.lib().dph_event_destroy(self.h)
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass


def _attn_work(a, off, label, mult):
    B, T, H, p = a[off], a[off + 1], a[off + 2], a[off + 4]
    return label + ("_drop" if p > 0 else ""), mult * B * H * T * T * 64, "flop"


def _conv0_bytes(a):
    B, S, C = a[1], a[2], a[4]
    L0 = (S - 10) // 5 + 1
    return 2.0 * B * L0 * C + 2.0 * 4 * B * S   # the bf16 output (its gradient) once + the waveform twice


# Algorithmic work of the non-GEMM launches bench.py tabulates (the argument order of include/dphubert_hip.h):
# attention in FLOPs (forward 4 B H T^2 64: Q K^T and P V; backward 2.5x that: dV, dP, dQ, dK plus the recomputed
# S), the memory-bound kernels in bytes of the tensors they must read / write once.
SPAN_WORK = {
    "dph_attention_fwd": lambda a: _attn_work(a, 6, "attn_fwd", 4.0),
    "dph_attention_fwd_relpos": lambda a: _attn_work(a, 8, "attn_fwd_relpos", 4.0),
    "dph_attention_bwd": lambda a: _attn_work(a, 7, "attn_bwd", 10.0),
    "dph_attention_bwd_relpos": lambda a: _attn_work(a, 11, "attn_bwd_relpos", 10.0),
    "dph_conv0_gn_fwd": lambda a: ("conv0_gn_fwd", _conv0_bytes(a), "byte"),
    "dph_conv0_gn_bwd": lambda a: ("conv0_gn_bwd", _conv0_bytes(a), "byte"),
    # x, y bf16 (+ the scaled input)
    "dph_layernorm_fwd": lambda a: ("ln_fwd", a[7] * a[8] * (4.0 + 2.0 * (a[1] is not None)), "byte"),
    "dph_layernorm_fwd_x32": lambda a: ("ln_fwd", a[6] * a[7] * 6.0, "byte"),
    # dy, x, dx bf16 (+ the branch gradient written, + its stored pre-activation read)
    "dph_layernorm_bwd": lambda a: ("ln_bwd", a[9] * a[10] * (6.0 + 2.0 * (a[13] is not None) +
                                                            2.0 * (a[18] is not None)), "byte"),
    "dph_layernorm_bwd_res32": lambda a: ("ln_bwd", a[8] * a[9] * (10.0 + 4.0 * (a[10] is not None)), "byte"),
    # 30 B per updated parameter (optim.FusedAdamW sets the count): p, g, m, v read, p, m, v + bf16 image written
    "dph_adamw_step_img": lambda a: ("adamw", 30.0 * SPAN_HINT.get("adamw_params", 0), "byte"),
}
SPAN_HINT = {}

# GEMM role tag (bench.py's mfma_util_attn_ffn: north_star's utilisation bar over masked attention + FFN): the
# GEMMs launched inside a ``role("ffn")`` block -- FFN1 / FFN2 forward, their input and weight gradients -- are
# recorded with that role by the LaunchProfiler
ROLE = [None]


class role:
    def __init__(self, name):
        self.name = name

    def __enter__(self):
        self.prev, ROLE[0] = ROLE[0], self.name
        return self

    def __exit__(self, *exc):
        ROLE[0] = self.prev


def tagged(name):
    """Decorator: run the function inside ``role(name)``."""
    def deco(fn):
        def wrap(*a, **kw):
            with role(name):
                return fn(*a, **kw)
        wrap.__name__, wrap.__doc__ = fn.__name__, fn.__doc__
        return wrap
    return deco


class LaunchProfiler:
    """Brackets every GEMM launch with HIP events on the launch stream (used by bench.py to
    measure per-kernel average durations live; off by default).  Works eagerly and inside a HIP
    graph capture (the events become event-record nodes, read after the replay)."""

    active = None

    def __init__(self, by_shape: bool = False):
        self.records = []
        # every event this profiler handed out.  Inside a capture each one becomes an event-record node of the graph,
        # which hipGraphLaunch records on every replay: the event must outlive the graph.  A launch that fails after
        # its first event was recorded (the grouped weight-gradient GEMM returning DPH_EUNSUPPORTED and falling back
        # to per-layer launches) used to drop that event with its Python wrapper -> hipEventDestroy -> the next
        # replay recorded a freed event and segfaulted on the host (round 3, gpurun_out/r3_s25).  Owned here, no
        # event can be collected before the profiler (kept by Trainer with the profiled graph).
        self.events = []
        self.by_shape = by_shape   # key the summary by (kernel, M, N, K, batch, splits) -- diagnostics
        self.spans = []            # (label, work, unit, e0, e1) of the SPAN_WORK launches

    def event(self) -> "_Event":
        e = _Event()
        self.events.append(e)
        return e

    def __enter__(self):
        LaunchProfiler.active = self
        _lib.CALL_HOOK[0] = self._span
        return self

    def __exit__(self, *exc):
        LaunchProfiler.active = None
        _lib.CALL_HOOK[0] = None

    def _span(self, name, fn, args):
        wk = SPAN_WORK.get(name)
        if wk is None:
            return fn(*args)
        e0, e1 = self.event(), self.event()
        e0.record()
        rc = fn(*args)
        e1.record()
        label, work, unit = wk(args)
        self.spans.append((label, float(work), unit, e0, e1))
        return rc

    def span_summary(self):
        """{label: {launches, ms, work, unit}} of the bracketed non-GEMM launches."""
        torch.cuda.synchronize()
        out = {}
        for label, work, unit, e0, e1 in self.spans:
            d = out.setdefault(label, {"launches": 0, "ms": 0.0, "work": 0.0, "unit": unit})
            d["launches"] += 1
            d["ms"] += e0.elapsed_time(e1)
            d["work"] += work
        return out

    def role_summary(self):
        """{role: {launches, ms, flops}} of the GEMM launches recorded inside a ``role`` block."""
        torch.cuda.synchronize()
        out = {}
        for name, flops, e0, e1, byt, rl in self.records:
            if rl is None:
                continue
            d = out.setdefault(rl, {"launches": 0, "ms": 0.0, "flops": 0.0})
            d["launches"] += 1
            d["ms"] += e0.elapsed_time(e1)
            d["flops"] += flops
        return out

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, flops, e0, e1, byt, _rl in self.records:
            ms = e0.elapsed_time(e1)
            d = out.setdefault(name, {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0})
            d["launches"] += 1
            d["ms"] += ms
            d["flops"] += flops
            d["bytes"] += byt
        return out


def _variant(args):
    """Name of the kernel dph_gemm launches for these args (matches rocprof kernel names)."""
    return _lib.lib().dph_gemm_variant(C.byref(args)).decode()


GEMM_NO_PERSIST = 1            # DphGemmArgs.flags (include/dphubert_hip.h)
GEMM_PRE_DGK = 2               # ACT_GELU: pre_out stores gelu'(pre)*colmask*keep/(1-p) (ACT_GELU_BWD_DGK's aux)
GEMM_RESID_F32 = 4             # the residual is fp32 (the pre-norm residual stream); set from the tensor's dtype
_SHARED_GPU = [0]


class shared_gpu:
    """GEMMs launched inside the block share the GPU with another stream's kernels (the teacher forward
    next to the student forward): they get one tile per block instead of the persistent ring grid."""

    def __enter__(self):
        _SHARED_GPU[0] += 1
        return self

    def __exit__(self, *exc):
        _SHARED_GPU[0] -= 1


# ops.deferred_reductions: while set, the list that keeps every column-sum workspace alive until the queued
# reductions that read it are flushed
KEEP_WS = [None]
# True inside an armed deferral scope (ops._Armed): only then can a call's slab be queued, so only then is it kept
ARMED = [False]


def _sk_scratch(args, dev):
    """Stream-K route (dph_gemm_sk_plan): the fp32 partial-tile buffer (stream-ordered caching allocator: reused only
    by work queued after this GEMM) and the hand-off flags, which must be zero at launch -- a fresh slice of the zero
    arena (ops.zeros_f32: re-zeroed by the graph's fill node on every replay; the teacher's side stream has its own
    arena).  Returns the tensors to keep alive until the launch is enqueued (None: not taken)."""
    if os.environ.get("DPH_GEMM_SK", "0")[:1] in ("", "0"):   # (opt-in route: no planning call per GEMM otherwise)
        return None
    nb, nf = C.c_int64(0), C.c_int64(0)
    if not _lib.lib().dph_gemm_sk_plan(C.byref(args), C.byref(nb), C.byref(nf)):
        return None
    from . import ops
    dev = dev if dev is not None else "cuda"
    ws = torch.empty(nb.value // 4, dtype=torch.float32, device=dev)
    fl = ops.zeros_f32(int(nf.value), dev)
    args.sk_ws, args.sk_ws_bytes = ws.data_ptr(), nb.value
    args.sk_flags, args.sk_nflags = fl.data_ptr(), nf.value
    return ws, fl


def gemm(A: DphMat, B: DphMat, Cm: DphMat, M: int, N: int, K: int, *, a_kcontig: bool, b_kcontig: bool,
         c_dtype: int = OUT_BF16, act: int = ACT_NONE, alpha: float = 1.0, batch: int = 1, splits: int = 1,
         bias=None, colmask=None, smask=None, vec_z_inner: int = 0, pre_out=None, aux_in=None, residual=None,
         colsum_out=None, colsum_aux=None, row_len=None, len_rows: int = 0, dropout_p: float = 0.0, seed: int = 0,
         drop_row_offset: int = 0, colsum_n: int = 0, device=None, flags: int = 0, dyn=None):
    """``dyn``: (int32 device tensor, offset) of a {m, n, k} device-side extent triplet (DphGemmArgs.dyn_ext)."""
    if residual is not None and residual.dtype == F32:
        flags |= GEMM_RESID_F32
    ws = None
    ws_bytes = 0
    if splits > 1:
        # fp32 slices (+ one ticket per 128x128 output tile for the in-launch split-K combine, opt-in:
        # the last-arriving block's serial slab sum measured 27.9 vs 26.0 ms per step)
        tiles = ((M + 127) // 128) * ((N + 127) // 128) * batch if _SPLITK_INLAUNCH else 0
        n_el = batch * splits * M * N + tiles
        ws_bytes = n_el * 4
        ws = torch.empty(n_el, dtype=F32, device=device or "cuda")
    elif (colsum_out is not None or colsum_aux is not None) and (batch == 1 or vec_z_inner == 0):
        # per-wave column-sum slab [2][batch][ceil(M/64)][N] (dph_gemm sums it in a fixed order instead of
        # same-address atomics)
        n_el = 2 * batch * ((M + 63) // 64) * N
        ws_bytes = n_el * 4
        ws = torch.empty(n_el, dtype=F32, device=device or Cm_device(colsum_out, colsum_aux))
        if KEEP_WS[0] is not None and ARMED[0]:
            KEEP_WS[0].append(ws)
    args = DphGemmArgs(M, N, K, batch, splits, int(a_kcontig), int(b_kcontig), A, B, Cm, c_dtype, act, alpha,
                       dropout_p, seed & 0xFFFFFFFFFFFFFFFF, ptr(bias), ptr(colmask), ptr(smask), vec_z_inner,
                       ptr(pre_out), ptr(aux_in), ptr(residual), ptr(colsum_out), ptr(colsum_aux), ptr(row_len),
                       len_rows, drop_row_offset, ptr(ws), ws_bytes, colsum_n,
                       flags | (GEMM_NO_PERSIST if _SHARED_GPU[0] else 0),
                       (dyn[0].data_ptr() + 4 * dyn[1]) if dyn is not None else None)
    sk_keep = _sk_scratch(args, device or Cm_device(colsum_out, colsum_aux))
    prof = LaunchProfiler.active
    if prof is not None:
        e0, e1 = prof.event(), prof.event()
        e0.record()
    call("dph_gemm", C.byref(args), _stream())
    del sk_keep
    if prof is not None:
        e1.record()
        name = _variant(args)
        if prof.by_shape:
            al = min((x & -x) if x else 1 << 20 for x in (Cm.ptr or 0, ptr(pre_out) or 0, ptr(aux_in) or 0,
                                                            ptr(residual) or 0, ptr(bias) or 0))
            name = (f"{name} M={M} N={N} K={K} b={batch} s={splits} {int(a_kcontig)}{int(b_kcontig)} act={act} "
                    f"res={residual is not None} rl={row_len is not None} rpbA={A.rows_per_batch} "
                    f"rsC={Cm.row_stride} align={al}")
        # algorithmic HBM bytes: A, B and C once, plus every epilogue operand the call reads or writes
        ob = 2 if c_dtype == OUT_BF16 else (8 if c_dtype == OUT_F32_ACCUM else 4)
        byt = batch * (2.0 * (M * K + N * K) + ob * M * N)
        for t, rw in ((pre_out, 1), (aux_in, 1), (residual, 1)):
            if t is not None:
                byt += rw * batch * M * N * t.element_size()
        prof.records.append((name, 2.0 * M * N * K * batch, e0, e1, byt, ROLE[0]))
    return ws  # keep alive until the stream consumes it (caching allocator is stream-ordered)


def Cm_device(*ts):
    for t in ts:
        if t is not None:
            return t.device
    return "cuda"


def choose_splits(M: int, N: int, K: int, batch: int = 1, target_blocks: int = 512) -> int:
    """Split-K factor of an (mn, mn) weight-gradient GEMM: the ping-pong kernel's tile / split plan
    (dph_gemm_mn_plan), else enough 128x128 register-staged blocks to fill the 256 CUs."""
    s = _lib.lib().dph_gemm_mn_plan(M, N, K, batch)
    if s > 0:
        return int(s)
    tiles = ((M + 127) // 128) * ((N + 127) // 128) * batch
    if tiles >= 256:
        return 1
    s = max(1, min(target_blocks // max(tiles, 1), K // 256))
    return int(s)


def linear_fwd(x: torch.Tensor, w_bf16: torch.Tensor, bias: Optional[torch.Tensor] = None, *, out=None,
               out_dtype=BF16, act=ACT_NONE, pre_out=None, colmask=None, smask=None, residual=None,
               dropout_p=0.0, seed=0, row_len=None, len_rows=0, colsum_out=None, pre_dgk=False, dyn=None):
    """y = epi(x @ w^T + b); x [M,K] bf16, w [N,K] bf16 (nn.Linear layout).

    ``pre_dgk`` (act=ACT_GELU): pre_out receives gelu'(pre)*colmask*keep/(1-p), the aux input of the matching
    ACT_GELU_BWD_DGK input-gradient GEMM, instead of the pre-activation."""
    _chk(x, BF16, "x")
    _chk(w_bf16, BF16, "w")
    M, K = x.shape
    N = w_bf16.shape[0]
    if out is None:
        # (an fp32 residual -- the pre-norm residual stream -- keeps its sum in fp32)
        dt = F32 if (residual is not None and residual.dtype == F32) else out_dtype
        out = torch.empty(M, N, dtype=dt, device=x.device)
    c_dtype = OUT_BF16 if out.dtype == BF16 else OUT_F32
    gemm(dense(x), dense(w_bf16), dense(out), M, N, K, a_kcontig=True, b_kcontig=True, c_dtype=c_dtype, act=act,
         bias=bias, colmask=colmask, smask=smask, pre_out=pre_out, residual=residual, dropout_p=dropout_p,
         seed=seed, row_len=row_len, len_rows=len_rows, colsum_out=colsum_out,
         flags=GEMM_PRE_DGK if pre_dgk else 0, dyn=dyn)
    return out


def linear_dgrad(dy: torch.Tensor, w_bf16: torch.Tensor, *, out=None, residual=None, act=ACT_NONE, aux_in=None,
                 colmask=None, colsum_out=None, colsum_aux=None, dropout_p=0.0, seed=0, colsum_n=0, w_t=None, dyn=None):
    """dx = epi(dy @ w); dy [M,N] bf16, w [N,K] bf16 -> [M,K] bf16 (fp32 with an fp32 ``out`` / ``residual``).

    ``w_t``: the [K,N] transposed image of w (ops.t_image): both GEMM operands are then
    k-contiguous and the LDS-DMA ring kernels take the GEMM."""
    M, N = dy.shape
    K = w_bf16.shape[1]
    if out is None:
        dt = F32 if (residual is not None and residual.dtype == F32) else BF16
        out = torch.empty(M, K, dtype=dt, device=dy.device)
    if w_t is not None:
        if tuple(w_t.shape) != (K, N):
            raise ValueError(f"w_t must be [{K},{N}], got {tuple(w_t.shape)}")
        B, bk = dense(w_t), True
    else:
        B, bk = dense(w_bf16), False
    gemm(dense(dy), B, dense(out), M, K, N, a_kcontig=True, b_kcontig=bk, residual=residual, act=act,
         c_dtype=OUT_BF16 if out.dtype == BF16 else OUT_F32,
         aux_in=aux_in, colmask=colmask, colsum_out=colsum_out, colsum_aux=colsum_aux, dropout_p=dropout_p,
         seed=seed, colsum_n=colsum_n, dyn=dyn)
    return out


def linear_wgrad(dy: torch.Tensor, x: torch.Tensor, dw: torch.Tensor, accumulate: bool = True, n_out: int = 0,
                 k_in: int = 0, dyn=None):
    """dw (+)= dy^T @ x; dy [M,N] bf16, x [M,K] bf16, dw [N,K] fp32.

    ``n_out`` / ``k_in`` < the operands' widths: only the first n_out x k_in block is produced
    (dy / x rows padded to multiples of 8 for pruned students; dw stays dense [n_out][k_in])."""
    M, N = dy.shape
    K = x.shape[1]
    Nw, Kw = (n_out or N), (k_in or K)
    splits = choose_splits(Nw, Kw, M)
    ws = gemm(dense(dy), dense(x), mat(dw, Kw), Nw, Kw, M, a_kcontig=False, b_kcontig=False,
              c_dtype=OUT_F32_ACCUM if accumulate else OUT_F32, splits=splits, device=dy.device, dyn=dyn)
    return ws


EUNSUPPORTED = -3


def linear_wgrad_grouped(items: Sequence, accumulate: bool = True) -> Optional[torch.Tensor]:
    """dw_i (+)= dy_i^T @ x_i for up to 16 problems of ONE shape in one launch (dph_gemm_grouped): the weight
    gradients of a group of encoder layers, whose blocks together fill the CUs that one layer's GEMM leaves idle
    without split-K.  ``items``: (dy [M,N] bf16, x [M,K] bf16, dw [N,K] fp32) triples.  Falls back to one
    linear_wgrad per problem where the grouped kernel does not apply (returns None then)."""
    n = len(items)
    if n == 0:
        return None
    dy0, x0, dw0 = items[0]
    M, N = dy0.shape
    K = x0.shape[1]
    ok = n <= _lib.GEMM_GROUP_MAX and all(
        tuple(dy.shape) == (M, N) and tuple(x.shape) == (M, K) and tuple(dw.shape) == (N, K) and
        dy.dtype == BF16 and x.dtype == BF16 and dw.dtype == F32 and dy.is_contiguous() and x.is_contiguous() and
        dw.stride() == (K, 1) for dy, x, dw in items)
    if not ok:
        for dy, x, dw in items:
            linear_wgrad(dy, x, dw, accumulate=accumulate)
        return None
    splits = choose_splits(N, K, M, batch=n)
    if splits == 1 and any(dw.data_ptr() % 16 for _, _, dw in items):
        # (the grouped kernel stores whole 16-byte vectors into each output)
        for dy, x, dw in items:
            linear_wgrad(dy, x, dw, accumulate=accumulate)
        return None
    ws, ws_bytes = None, 0
    if splits > 1:
        ws = torch.empty(n * splits * N * K, dtype=F32, device=dy0.device)
        ws_bytes = ws.numel() * 4
    args = DphGemmArgs(N, K, M, n, splits, 0, 0, dense(dy0), dense(x0), mat(dw0, K),
                       OUT_F32_ACCUM if accumulate else OUT_F32, ACT_NONE, 1.0, 0.0, 0, None, None, None, 0, None,
                       None, None, None, None, None, 0, 0, ptr(ws), ws_bytes, 0, 0, None)
    grp = _lib.DphGemmGroup()
    grp.n = n
    for i, (dy, x, dw) in enumerate(items):
        grp.a[i], grp.b[i], grp.c[i] = dy.data_ptr(), x.data_ptr(), dw.data_ptr()
    prof = LaunchProfiler.active
    if prof is not None:
        e0, e1 = prof.event(), prof.event()   # (owned by the profiler: e0 is recorded even if the launch falls back)
        e0.record()
    if _lib.TRACE[0]:
        with torch.profiler.record_function("dph::dph_gemm_grouped"):
            rc = _lib.lib().dph_gemm_grouped(C.byref(args), C.byref(grp), _stream())
    else:
        rc = _lib.lib().dph_gemm_grouped(C.byref(args), C.byref(grp), _stream())
    if rc == EUNSUPPORTED:
        for dy, x, dw in items:
            linear_wgrad(dy, x, dw, accumulate=accumulate)
        return None
    _lib.check(rc, "dph_gemm_grouped")
    if prof is not None:
        e1.record()
        name = _variant(args)
        if prof.by_shape:
            name = f"{name} grouped M={N} N={K} K={M} b={n} s={splits}"
        prof.records.append((name, 2.0 * M * N * K * n, e0, e1, n * (2.0 * (M * N + M * K) + 8.0 * N * K), ROLE[0]))
    return ws
