"""ctypes binding of the C ABI in include/dphubert_hip.h.

This is the "reference-side binding" of the boundary: plain pointers, sizes
and the current HIP stream go in, an int status comes back.  There is no
fallback: if the library is missing or a call fails, a RuntimeError is raised
(the product path never silently degrades to PyTorch/CPU math).
"""

import ctypes as C
import os
from pathlib import Path

import torch

_HERE = Path(__file__).resolve().parent
# DPH_LIB_PATH selects another build of the same library (A/B measurements)
LIB_PATH = Path(os.environ.get("DPH_LIB_PATH", str(_HERE / "libdphubert_hip.so")))

vp = C.c_void_p
i64 = C.c_int64
i32 = C.c_int32
f32 = C.c_float
u64 = C.c_uint64


class DphMat(C.Structure):
    _fields_ = [("ptr", vp), ("rows_per_batch", i64), ("batch_stride", i64), ("row_stride", i64),
                ("z_div", i64), ("z_outer", i64), ("z_inner", i64)]


class DphGemmArgs(C.Structure):
    _fields_ = [("M", i64), ("N", i64), ("K", i64), ("batch", i32), ("splits", i32), ("a_kcontig", i32),
                ("b_kcontig", i32), ("A", DphMat), ("B", DphMat), ("C", DphMat), ("c_dtype", i32), ("act", i32),
                ("alpha", f32), ("dropout_p", f32), ("seed", u64), ("bias", vp), ("colmask", vp), ("smask", vp),
                ("vec_z_inner", i64), ("pre_out", vp), ("aux_in", vp), ("residual", vp), ("colsum_out", vp),
                ("colsum_aux", vp), ("row_len", vp), ("len_rows", i64), ("drop_row_offset", i64),
                ("workspace", vp), ("workspace_bytes", i64), ("colsum_n", i64), ("flags", i64), ("dyn_ext", vp),
                ("sk_ws", vp), ("sk_ws_bytes", i64), ("sk_flags", vp), ("sk_nflags", i64)]


GEMM_GROUP_MAX = 16


class DphGemmGroup(C.Structure):
    _fields_ = [("n", i32), ("reserved", i32), ("a", vp * GEMM_GROUP_MAX), ("b", vp * GEMM_GROUP_MAX),
                ("c", vp * GEMM_GROUP_MAX)]


class DphTensorSlot(C.Structure):
    _fields_ = [("param", vp), ("grad", vp), ("exp_avg", vp), ("exp_avg_sq", vp), ("n", i64), ("group", i32),
                ("pad_", i32)]


class DphAdamGroup(C.Structure):
    _fields_ = [("lr", f32), ("weight_decay", f32), ("beta1", f32), ("beta2", f32), ("eps", f32),
                ("pad_", f32 * 3)]


class DphAdamDyn(C.Structure):
    _fields_ = [("g", DphAdamGroup * 4), ("step", f32), ("pad_", f32 * 3)]


class DphHcEntry(C.Structure):
    _fields_ = [("log_alpha", vp), ("u_in", vp), ("dmask", vp), ("dlog_alpha", vp), ("n", i64), ("offset", i64)]


S = vp  # hipStream_t

_SIGS = {
    "dph_abi_version": ([], C.c_int),
    "dph_set_deterministic": ([C.c_int], C.c_int),
    "dph_get_deterministic": ([], C.c_int),
    "dph_defer_reductions": ([C.c_int], C.c_int),
    "dph_flush_reductions": ([S], C.c_int),
    "dph_deferred_reductions": ([], i64),
    "dph_discard_reductions": ([], i64),
    "dph_gemm_sk_plan": ([C.POINTER(DphGemmArgs), C.POINTER(i64), C.POINTER(i64)], C.c_int),
    "dph_reductions_pushed": ([], i64),
    "dph_gemm": ([C.POINTER(DphGemmArgs), S], C.c_int),
    "dph_gemm_mn_plan": ([i64, i64, i64, i64], C.c_int),
    "dph_gemm_grouped": ([C.POINTER(DphGemmArgs), C.POINTER(DphGemmGroup), S], C.c_int),
    "dph_ffn_compact": ([vp, i64, i64, vp, vp, S], C.c_int),
    "dph_ffn_pack": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, i64, S], C.c_int),
    "dph_ffn_unpack_grads": ([vp, vp, vp, vp, vp, vp, i64, vp, vp, vp, i64, i64, S], C.c_int),
    "dph_gather_rows_bf16": ([vp, i64, vp, vp, i64, i64, S], C.c_int),
    "dph_gather_cols_bf16": ([vp, i64, vp, vp, i64, i64, S], C.c_int),
    "dph_gather_vec_f32": ([vp, vp, vp, i64, S], C.c_int),
    "dph_scatter_rows_f32": ([vp, vp, vp, i64, i64, i64, C.c_int, S], C.c_int),
    "dph_scatter_cols_f32": ([vp, vp, vp, i64, i64, i64, C.c_int, S], C.c_int),
    "dph_layernorm_fwd": ([vp, vp, vp, vp, vp, vp, vp, i64, i64, f32, f32, u64, S], C.c_int),
    "dph_layernorm_bwd": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, f32, u64, vp, f32, u64, vp, vp, vp, vp, vp, i64,
                           S],
                          C.c_int),
    "dph_layernorm_fwd_ld": ([vp, vp, vp, vp, vp, vp, vp, i64, i64, i64, f32, f32, u64, S], C.c_int),
    "dph_layernorm_bwd_ld": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, i64, f32, u64, vp, f32, u64, vp, vp, vp,
                              vp, vp, vp, i64, S], C.c_int),
    "dph_wave_layernorm": ([vp, vp, i64, i64, f32, vp, S], C.c_int),
    "dph_colsum": ([vp, vp, i64, i64, vp, i64, S], C.c_int),
    "dph_colsum3": ([vp, vp, vp, vp, i64, i64, vp, i64, S], C.c_int),
    "dph_colsum_workspace": ([i64, i64], i64),
    "dph_colprod": ([vp, i64, vp, i64, vp, vp, i64, i64, S], C.c_int),
    "dph_layernorm_bwd_workspace": ([i64, i64], i64),
    "dph_attention_fwd": ([vp, vp, vp, vp, vp, vp, i64, i64, i64, f32, f32, u64, vp, S], C.c_int),
    "dph_attention_keep_bytes": ([i64, i64, i64], i64),
    "dph_attention_bwd_prep": ([vp, vp, vp, vp, vp, i64, i64, i64, vp, i64, S], C.c_int),
    "dph_attention_bwd_prep_workspace": ([i64, i64, i64], i64),
    "dph_attention_bwd": ([vp, vp, vp, vp, vp, vp, vp, i64, i64, i64, f32, f32, u64, vp, S], C.c_int),
    "dph_attention_bwd_qv": ([vp, vp, vp, vp, vp, vp, vp, i64, i64, i64, f32, f32, u64, vp, vp, vp, vp, i64, S],
                             C.c_int),
    "dph_attention_bwd_qv_workspace": ([i64, i64, i64], i64),
    "dph_attention_fwd_relpos": ([vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, i64, f32, f32, u64, vp, S], C.c_int),
    "dph_attention_bwd_relpos": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, i64, f32, f32, u64, vp, vp,
                                  i64, S], C.c_int),
    "dph_attention_bwd_relpos_workspace": ([i64, i64, i64], i64),
    "dph_attention_bwd_relpos_qv": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, i64, f32, f32, u64, vp, vp,
                                     i64, vp, vp, vp, i64, S], C.c_int),
    "dph_relpos_table": ([vp, vp, vp, vp, i64, i64, i64, i64, i64, S], C.c_int),
    "dph_relpos_table_bwd": ([vp, vp, vp, i64, i64, i64, i64, i64, S], C.c_int),
    "dph_wavlm_gate_fwd": ([vp, i64, vp, vp, vp, vp, vp, i64, i64, i64, i64, S], C.c_int),
    "dph_wavlm_gate_bwd": ([vp, i64, vp, vp, vp, vp, vp, vp, i64, vp, vp, vp, vp, i64, i64, i64, i64, i64, S],
                           C.c_int),
    "dph_wavlm_gate_bwd_workspace": ([i64, i64, i64], i64),
    "dph_conv0_gn_fwd": ([vp, i64, i64, vp, i64, i64, i64, vp, vp, vp, vp, vp, vp, vp, i64, S], C.c_int),
    "dph_conv0_gn_bwd_workspace": ([i64, i64, i64], i64),
    "dph_conv0_bwd_workspace": ([i64, i64, i64], i64),
    "dph_conv0_gn_bwd": ([vp, i64, i64, vp, i64, i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, S],
                         C.c_int),
    "dph_conv0_fwd": ([vp, i64, i64, vp, vp, i64, i64, i64, vp, S], C.c_int),
    "dph_col2im_gelu_bwd": ([vp, i64, i64, i64, i64, i64, i64, vp, vp, vp, vp, vp, i64, S], C.c_int),
    "dph_gelu_mask_bwd": ([vp, vp, vp, vp, vp, i64, i64, vp, i64, S], C.c_int),
    "dph_rowblock_workspace": ([i64, i64], i64),
    "dph_regroup_pad": ([vp, vp, i64, i64, i64, i64, i64, i64, S], C.c_int),
    "dph_weight_norm_fwd": ([vp, vp, i64, i64, i64, i64, vp, vp, vp, vp, vp, i64, S], C.c_int),
    "dph_weight_norm_bwd": ([vp, vp, vp, vp, i64, i64, i64, i64, vp, vp, vp, i64, S], C.c_int),
    "dph_cast_bf16": ([vp, vp, i64, S], C.c_int),
    "dph_transpose_bf16": ([vp, i64, i64, vp, S], C.c_int),
    "dph_cast_bf16_multi": ([vp, i64, S], C.c_int),
    "dph_copy_f32_multi": ([vp, i64, i64, S], C.c_int),
    "dph_conv_lengths": ([vp, vp, i64, i64, vp, vp, S], C.c_int),
    "dph_conv0_bwd": ([vp, i64, i64, i64, i64, i64, vp, vp, vp, vp, i64, S], C.c_int),
    "dph_gelu_mask_fwd": ([vp, vp, vp, i64, i64, S], C.c_int),
    "dph_layernorm_gelu_fwd": ([vp, C.c_int, vp, vp, vp, vp, vp, vp, vp, i64, i64, f32, S], C.c_int),
    "dph_layernorm_bwd_x32": ([vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, vp, i64, S], C.c_int),
    "dph_transpose_bf16_multi": ([vp, i64, S], C.c_int),
    "dph_layernorm_fwd_x32": ([vp, vp, vp, vp, vp, vp, i64, i64, f32, S], C.c_int),
    "dph_layernorm_bwd_res32": ([vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, vp, vp, i64, S], C.c_int),
    "dph_branch_bwd_f32": ([vp, vp, C.c_int, i64, i64, f32, u64, vp, vp, i64, vp, vp, vp, vp, i64, S], C.c_int),
    "dph_conv_weight_pack": ([vp, vp, i64, i64, i64, i64, i64, S], C.c_int),
    "dph_conv_weight_unpack_grad": ([vp, vp, i64, i64, i64, i64, C.c_int, S], C.c_int),
    "dph_add_bf16": ([vp, vp, vp, i64, S], C.c_int),
    "dph_branch_bwd": ([vp, vp, i64, i64, f32, u64, vp, vp, i64, vp, vp, vp, vp, i64, S], C.c_int),
    "dph_distill_loss_fwd": ([vp, vp, i64, i64, i64, i64, f32, f32, f32, C.c_int, vp, vp, vp, S], C.c_int),
    "dph_distill_loss_bwd": ([vp, vp, vp, vp, i64, i64, i64, i64, f32, f32, f32, C.c_int, vp, S], C.c_int),
    "dph_distill_loss_fwd_ex": ([vp, vp, C.c_uint32, i64, i64, i64, i64, f32, f32, f32, C.c_int, vp, vp, vp, S],
                                C.c_int),
    "dph_distill_loss_bwd_ex": ([vp, vp, C.c_uint32, vp, vp, i64, i64, i64, i64, f32, f32, f32, C.c_int, vp, S],
                                C.c_int),
    "dph_reg_loss_fwd": ([vp, vp, vp, vp, vp, f32, f32, vp, S], C.c_int),
    "dph_reg_loss_bwd": ([vp, vp, vp, vp, vp, vp, vp, f32, f32, vp, vp, vp, S], C.c_int),
    "dph_hc_sample_fwd": ([vp, vp, vp, vp, i64, u64, f32, f32, f32, f32, S], C.c_int),
    "dph_hc_sample_bwd": ([vp, vp, vp, vp, i64, f32, f32, f32, S], C.c_int),
    "dph_hc_bank_fwd": ([vp, i64, vp, vp, u64, f32, f32, f32, f32, S], C.c_int),
    "dph_hc_bank_bwd": ([vp, i64, vp, f32, f32, f32, S], C.c_int),
    "dph_expected_params_fwd": ([vp, vp, i64, vp, vp, i64, C.c_double, f32, vp, vp, S], C.c_int),
    "dph_expected_params_bwd": ([vp, vp, vp, vp, i64, vp, vp, i64, vp, vp, f32, S], C.c_int),
    "dph_grad_sumsq": ([vp, i64, vp, vp, i64, vp, S], C.c_int),
    "dph_adamw_step": ([vp, i64, vp, vp, i64, vp, i64, i64, vp, f32, S], C.c_int),
    "dph_adamw_step_dev": ([vp, i64, vp, vp, i64, vp, vp, f32, S], C.c_int),
    "dph_adamw_step_img": ([vp, i64, vp, vp, i64, vp, vp, i64, i64, vp, f32, vp, S], C.c_int),
    "dph_set_rng_epoch": ([vp], C.c_int),
    "dph_event_create": ([C.POINTER(vp)], C.c_int),
    "dph_event_record": ([vp, S], C.c_int),
    "dph_event_elapsed_ms": ([vp, vp, C.POINTER(f32)], C.c_int),
    "dph_event_destroy": ([vp], C.c_int),
}

_lib = None
# include/dphubert_hip.h layout (3: dph_adamw_step_dev, dph_set_rng_epoch; 4: dph_event_*; 5: LN bwd / colsum
# workspaces; 12: dph_hc_bank_fwd / dph_hc_bank_bwd; 15: dph_gemm_mn_plan; 16: DphGemmArgs.dyn_ext, dph_ffn_compact + gathers / scatters;
# 19: DPH_GEMM_RESID_F32, dph_layernorm_fwd_x32 / _bwd_res32, dph_branch_bwd_f32, dph_distill_loss_*_ex: the fp32
# pre-norm residual stream; 20: deterministic mode -- dph_set_deterministic / dph_get_deterministic and the workspaces
# of the fixed-order reductions: attention prep / relpos backward, WavLM gate, conv0, GELU-mask and branch backward;
# 21: deferred column reductions -- dph_defer_reductions / dph_flush_reductions / dph_deferred_reductions;
# 22: dph_attention_bwd_prep's D is the rowdot of dO_m itself, the head mask applied to dq / dk / dv in fp32;
# 23: dph_discard_reductions / dph_reductions_pushed, queue-flush launch errors propagated by every column reduction;
#     DphGemmArgs.sk_* + dph_gemm_sk_plan: the persistent stream-K 256 x 256 GEMM;
# 24: dph_attention_bwd_qv / dph_attention_bwd_relpos_qv + dph_attention_bwd_qv_workspace: the q / v bias
#     gradients summed inside the attention backward)
ABI_VERSION = 24


class DphError(RuntimeError):
    pass


def lib():
    """Load the kernel library (raises if it is missing: no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise DphError(f"{LIB_PATH} not found: run `python -m dphubert_amd.build` (hipcc --offload-arch=gfx950)")
    L = C.CDLL(str(LIB_PATH))
    L.dph_last_error.restype = C.c_char_p
    L.dph_last_error.argtypes = []
    if hasattr(L, "dph_gemm_variant"):
        L.dph_gemm_variant.restype = C.c_char_p
        L.dph_gemm_variant.argtypes = [C.POINTER(DphGemmArgs)]
    missing = []
    for name, (args, res) in _SIGS.items():
        try:
            fn = getattr(L, name)
        except AttributeError:
            missing.append(name)
            continue
        fn.argtypes = args
        fn.restype = res
    L.missing_symbols = missing
    if "dph_abi_version" not in missing and L.dph_abi_version() != ABI_VERSION:
        raise DphError(f"{LIB_PATH}: ABI {L.dph_abi_version()} != {ABI_VERSION}; rebuild (python -m dphubert_amd.build)")
    _lib = L
    return L


def exported_symbols():
    return ["dph_last_error", "dph_gemm_variant"] + list(_SIGS)


def set_deterministic(on: bool = True) -> None:
    """Process-wide deterministic mode of the kernel library (include/dphubert_hip.h): fixed-order cross-block
    reductions instead of float atomics, so repeated runs of a step (eager or replayed) are bitwise identical.
    Set it before capturing a HIP graph (a captured graph keeps the kernels it recorded)."""
    check(lib().dph_set_deterministic(1 if on else 0), "dph_set_deterministic")


def deterministic() -> bool:
    return bool(lib().dph_get_deterministic())


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().dph_last_error().decode(errors="replace")
        raise DphError(f"{what or 'dph call'} failed ({rc}): {msg}")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


# set by kernels.LaunchProfiler while it is active: brackets the non-GEMM launches its table covers
CALL_HOOK = [None]


# Tracing (SURVEY 5 "Tracing / profiling"): with DPH_TRACE=1 (or set_trace(True)) every C-ABI call runs inside a
# torch.profiler.record_function range named after the entry point, so a torch.profiler / Kineto trace shows which
# library call enqueued each HIP kernel next to the reference's module names.  Off by default: a range costs a few
# microseconds of host time per call (there are ~600 calls in an eager step).  Inside a HIP-graph capture the ranges
# mark the capture, not the replays.
TRACE = [os.environ.get("DPH_TRACE", "0") == "1"]


def set_trace(on: bool) -> bool:
    prev, TRACE[0] = TRACE[0], bool(on)
    return prev


def call(name: str, *args):
    fn = getattr(lib(), name)
    hook = CALL_HOOK[0]
    if TRACE[0]:
        with torch.profiler.record_function(f"dph::{name}"):
            rc = hook(name, fn, args) if hook is not None else fn(*args)
    else:
        rc = hook(name, fn, args) if hook is not None else fn(*args)
    check(rc, name)
