"""The LayerNorm kernels directly against a plain PyTorch fp32 LayerNorm (components.py:846-856 pre-/post-norm,
model.py LayerNorm over the residual stream), every entry point the layers call:

  * dph_layernorm_fwd / _bwd_ld: bf16 x / dx (post-norm), dx_add (bf16);
  * dph_layernorm_fwd_x32 / _bwd_x32 / _bwd_res32: the fp32 residual stream (pre-norm, Large), fp32 dx + dx_add;

at the widths the 16-byte half-wave kernels take (D = 256 k <= 1024), one they do not (384, the 8-byte quad
kernels), ragged row counts (1, 37: a partial block and a partial wave) and a misaligned base pointer (the quad
fallback).  Tolerances: bf16 outputs rtol 1e-2 / atol 2e-2 (one bf16 rounding of O(1) values); fp32 outputs
rtol 1e-4 / atol 1e-4 (the kernels compute in fp32 from the same bf16 dy); dgamma / dbeta are sums over the rows
(atol scaled by sqrt(rows))."""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
EPS = 1e-5


def _inputs(rows, D, xdt, seed, misalign=False):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = (torch.randn(rows, D, generator=g) * 1.7 + 0.3)
    dy = torch.randn(rows, D, generator=g).to(torch.bfloat16)
    gamma = torch.rand(D, generator=g) + 0.5
    beta = torch.randn(D, generator=g) * 0.1
    add = torch.randn(rows, D, generator=g)
    if misalign:
        # same values, base pointer 8 bytes past a 16-byte boundary (bf16 only: the fp32 quad kernels load float4)
        buf = torch.empty(rows * D + 4, dtype=xdt, device=DEV)
        xd = buf[4:].view(rows, D)
        xd.copy_(x.to(xdt))
    else:
        xd = x.to(xdt).to(DEV)
    return xd, dy.to(DEV), gamma.to(DEV), beta.to(DEV), add.to(DEV)


def _ref(x, dy, gamma, beta):
    xr = x.float().clone().requires_grad_(True)
    w = gamma.clone().requires_grad_(True)
    b = beta.clone().requires_grad_(True)
    y = torch.nn.functional.layer_norm(xr, (x.shape[1],), w, b, EPS)
    y.backward(dy.float())
    mu = x.float().mean(1)
    rs = torch.rsqrt(x.float().var(1, unbiased=False) + EPS)
    return y.detach(), xr.grad, w.grad, b.grad, mu, rs


CASES = [(1, 256), (37, 768), (1000, 768), (1000, 1024), (300, 512), (37, 384)]


@pytest.mark.parametrize("rows,D", CASES)
@pytest.mark.parametrize("x32", [False, True])
@pytest.mark.parametrize("misalign", [False, True])
def test_layernorm_fwd_vs_torch(rows, D, x32, misalign):
    if misalign and x32:
        pytest.skip("fp32 rows stay 16-byte aligned")
    from dphubert_amd._lib import call, ptr, stream_ptr
    xdt = torch.float32 if x32 else torch.bfloat16
    x, dy, gamma, beta, _ = _inputs(rows, D, xdt, 11 + rows + D, misalign)
    y = torch.empty(rows, D, device=DEV, dtype=torch.bfloat16)
    mu = torch.empty(rows, device=DEV)
    rs = torch.empty(rows, device=DEV)
    if x32:
        call("dph_layernorm_fwd_x32", ptr(x), ptr(gamma), ptr(beta), ptr(y), ptr(mu), ptr(rs), rows, D, EPS,
             stream_ptr())
    else:
        call("dph_layernorm_fwd", ptr(x), None, ptr(gamma), ptr(beta), ptr(y), ptr(mu), ptr(rs), rows, D, EPS, 0.0,
             0, stream_ptr())
    torch.cuda.synchronize()
    yr, _, _, _, mur, rsr = _ref(x, dy, gamma, beta)
    torch.testing.assert_close(mu, mur, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(rs, rsr, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(y.float(), yr, rtol=1e-2, atol=2e-2)


def _ws(rows, D):
    from dphubert_amd import _lib
    n = _lib.lib().dph_layernorm_bwd_workspace(rows, D)
    return torch.empty(max(1, n // 4), device=DEV), n


@pytest.mark.parametrize("rows,D", CASES)
@pytest.mark.parametrize("kind", ["bf16", "bf16_add", "x32", "res32", "res32_add"])
@pytest.mark.parametrize("misalign", [False, True])
def test_layernorm_bwd_vs_torch(rows, D, kind, misalign):
    from dphubert_amd._lib import call, ptr, stream_ptr
    xdt = torch.bfloat16 if kind.startswith("bf16") else torch.float32
    if misalign and xdt == torch.float32:
        pytest.skip("fp32 rows stay 16-byte aligned")
    x, dy, gamma, beta, add = _inputs(rows, D, xdt, 23 + rows + D, misalign)
    mu = torch.empty(rows, device=DEV)
    rs = torch.empty(rows, device=DEV)
    y = torch.empty(rows, D, device=DEV, dtype=torch.bfloat16)
    if xdt == torch.float32:
        call("dph_layernorm_fwd_x32", ptr(x), ptr(gamma), ptr(beta), ptr(y), ptr(mu), ptr(rs), rows, D, EPS,
             stream_ptr())
    else:
        call("dph_layernorm_fwd", ptr(x), None, ptr(gamma), ptr(beta), ptr(y), ptr(mu), ptr(rs), rows, D, EPS, 0.0,
             0, stream_ptr())
    dxdt = torch.float32 if kind.startswith("res32") else torch.bfloat16
    dx = torch.empty(rows, D, device=DEV, dtype=dxdt)
    dw = torch.zeros(D, device=DEV)
    db = torch.zeros(D, device=DEV)
    ws, nws = _ws(rows, D)
    addt = add.to(dxdt) if kind.endswith("_add") else None
    if kind.startswith("bf16"):
        call("dph_layernorm_bwd_ld", ptr(dy), ptr(x), None, ptr(gamma), ptr(mu), ptr(rs), ptr(dx), ptr(dw), ptr(db),
             rows, D, D, 0.0, 0, None, 0.0, 0, None, None, None, None, ptr(addt) if addt is not None else None, ptr(ws),
             nws, stream_ptr())
    elif kind == "x32":
        call("dph_layernorm_bwd_x32", ptr(dy), ptr(x), ptr(gamma), ptr(mu), ptr(rs), ptr(dx), ptr(dw), ptr(db),
             rows, D, ptr(ws), nws, stream_ptr())
    else:
        call("dph_layernorm_bwd_res32", ptr(dy), ptr(x), ptr(gamma), ptr(mu), ptr(rs), ptr(dx), ptr(dw), ptr(db),
             rows, D, ptr(addt) if addt is not None else None, ptr(ws), nws, stream_ptr())
    torch.cuda.synchronize()
    _, dxr, dwr, dbr, _, _ = _ref(x, dy, gamma, beta)
    if addt is not None:
        dxr = dxr + addt.float()
    if dxdt == torch.float32:
        torch.testing.assert_close(dx, dxr, rtol=1e-4, atol=1e-4)
    else:
        torch.testing.assert_close(dx.float(), dxr, rtol=1e-2, atol=2e-2)
    tol = 1e-4 * math.sqrt(rows) + 1e-5
    torch.testing.assert_close(dw, dwr, rtol=1e-4, atol=tol)
    torch.testing.assert_close(db, dbr, rtol=1e-4, atol=tol)
