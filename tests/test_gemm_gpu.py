"""GEMM parity on the GPU: every operand layout and epilogue against a torch fp32
reference of the same op on the same bf16-rounded inputs."""

import pytest
import torch

pytestmark = pytest.mark.gpu

torch.manual_seed(0)


@pytest.fixture(autouse=True, params=["small", "mid", "big", "wide", "flat", "flat-np", "tall", "half", "mid8",
                                     "mid8mn", "tri", "tri-np", "pp256", "pp128x256", "pp256x128", "pp128x192", "pp128x192-nopf", "pp128", "ppw"])
def gemm_path(request, monkeypatch):
    """Run every test on each GEMM path: the 128x128 register-staged kernel and the 128x128 /
    256x256 / 256x128 / 128x256 / 256x64 / 192x128 LDS-DMA ring kernels (taken where their constraints hold: both operands
    k-contiguous, K % 32 == 0), and the ping-pong kernels (both operands k-contiguous, K % 64 == 0, K >= 128)."""
    path = request.param
    if path.endswith("-np"):            # one tile per block instead of the persistent grid
        monkeypatch.setenv("DPH_GEMM_PERSIST", "0")
        path = path[:-3]
    if path.endswith("-nopf"):          # one-round 128 x 192 grids on the plain schedule (no B-n0 prefetch)
        monkeypatch.setenv("DPH_PP_B0PF", "0")
        path = path[:-5]
    monkeypatch.setenv("DPH_GEMM_PATH", path)
    return request.param


def _k():
    from dphubert_amd import kernels as K
    return K


def rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device="cuda") * scale).to(torch.bfloat16)


def close(a, b, tol=2e-2):
    a = a.float()
    b = b.float()
    err = (a - b).norm() / b.norm().clamp_min(1e-20)
    assert err < tol, f"rel err {err}"


@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(304, 200, 136), (128, 128, 64), (1000, 264, 520), (1000, 264, 512),
                                   (2056, 520, 768), (256, 256, 64), (7984, 768, 192),
                                   (504, 48, 1536)])
def test_layouts(ak, bk, M, N, K):
    K_ = _k()
    A = rnd(M, K) if ak else rnd(K, M)
    B = rnd(N, K) if bk else rnd(K, N)
    Af = A.float() if ak else A.float().t()
    Bf = B.float().t() if bk else B.float()
    ref = Af @ Bf
    C = torch.empty(M, N, device="cuda", dtype=torch.float32)
    K_.gemm(K_.dense(A), K_.dense(B), K_.dense(C), M, N, K, a_kcontig=ak, b_kcontig=bk, c_dtype=K_.OUT_F32)
    torch.cuda.synchronize()
    close(C, ref, 1e-5)


def test_asymmetric_identity():
    # A = I with an asymmetric B catches a transposed C write (guide: A=I check)
    K_ = _k()
    M = N = K = 128
    A = torch.eye(M, device="cuda").to(torch.bfloat16)
    B = (torch.arange(N * K, device="cuda").reshape(N, K) % 251).to(torch.bfloat16)
    C = torch.empty(M, N, device="cuda")
    K_.gemm(K_.dense(A), K_.dense(B), K_.dense(C), M, N, K, a_kcontig=True, b_kcontig=True, c_dtype=K_.OUT_F32)
    torch.cuda.synchronize()
    assert torch.equal(C, B.float().t())


def test_epilogue_gelu_mask_pre():
    K_ = _k()
    M, N, K = 513, 384, 256
    x, w = rnd(M, K), rnd(N, K, scale=0.05)
    b = torch.randn(N, device="cuda")
    cm = torch.rand(N, device="cuda")
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    y = K_.linear_fwd(x, w, b, act=K_.ACT_GELU, pre_out=pre, colmask=cm)
    u = x.float() @ w.float().t() + b
    close(pre, u)
    close(y, torch.nn.functional.gelu(u) * cm)


def test_epilogue_residual_smask_colsum_rowlen():
    K_ = _k()
    M, N, K = 400, 256, 128
    x, w = rnd(M, K), rnd(N, K, scale=0.1)
    b = torch.randn(N, device="cuda")
    res = rnd(M, N)
    sm = torch.tensor([0.7], device="cuda")
    cs = torch.zeros(N, device="cuda")
    lens = torch.tensor([150, 200], device="cuda", dtype=torch.int64)
    y = K_.linear_fwd(x, w, b, smask=sm, residual=res, colsum_out=cs, row_len=lens, len_rows=200)
    ref = (x.float() @ w.float().t() + b) * 0.7 + res.float()
    ref[150:200] = 0
    close(y, ref)
    close(cs, y.float().sum(0), 1e-2)


def test_gelu_bwd_epilogue():
    K_ = _k()
    M, N, K = 300, 512, 192   # dF = dY @ W2 ; N = F
    dy, w2 = rnd(M, K), rnd(K, N, scale=0.05)    # W2 [D=K][F=N]
    u = rnd(M, N)
    im = torch.rand(N, device="cuda")
    dm = torch.zeros(N, device="cuda")
    db = torch.zeros(N, device="cuda")
    du = K_.linear_dgrad(dy, w2, act=K_.ACT_GELU_BWD, aux_in=u, colmask=im, colsum_out=db, colsum_aux=dm)
    df = dy.float() @ w2.float()
    uf = u.float().requires_grad_(True)
    g = torch.nn.functional.gelu(uf)
    gp, = torch.autograd.grad(g.sum(), uf)
    close(du, df * im * gp)
    close(dm, (df * g.detach()).sum(0), 1e-2)
    close(db, du.float().sum(0), 1e-2)


@pytest.mark.parametrize("accum", [False, True])
def test_wgrad_splitk(accum):
    K_ = _k()
    M, N, K = 3000, 384, 256
    dy, x = rnd(M, N), rnd(M, K)
    dw = torch.randn(N, K, device="cuda")
    dw0 = dw.clone()
    K_.linear_wgrad(dy, x, dw, accumulate=accum)
    ref = dy.float().t() @ x.float() + (dw0 if accum else 0)
    close(dw, ref, 1e-5)


@pytest.mark.parametrize("N,K,M", [(2304, 768, 7984), (768, 768, 7984), (768, 3072, 7984), (512, 1024, 3000),
                                   (200, 136, 1000)])
def test_wgrad_ppw_plan(N, K, M, gemm_path):
    """(mn, mn) weight gradients on the ping-pong kernel's own tile / split plan (dph_gemm_mn_plan): the
    step's projection shapes (K = B*T = 7984: a 48-row K tail), fp32 accumulation into an existing gradient."""
    K_ = _k()
    if gemm_path != "ppw":
        pytest.skip("ppw plan only")
    dy, x = rnd(M, N), rnd(M, K)
    dw = torch.randn(N, K, device="cuda")
    dw0 = dw.clone()
    assert "ppw_gemm_kernel" in K_._variant(_wgrad_args(K_, dy, x, dw))
    keep = K_.linear_wgrad(dy, x, dw, accumulate=True)
    torch.cuda.synchronize()
    del keep
    ref = dy.double().t() @ x.double() + dw0.double()
    close(dw, ref, 1e-5)


@pytest.mark.parametrize("n,N,K,M", [(6, 768, 768, 7984), (3, 2304, 768, 7984), (2, 768, 3072, 1000), (5, 200, 136, 1000),
                                     (16, 128, 64, 300)])
def test_wgrad_grouped(n, N, K, M, gemm_path):
    """dph_gemm_grouped: n independent (mn, mn) weight gradients of one shape in one launch (the deferred encoder
    layers' dW_i += dY_i^T X_i) against fp64 torch per problem; every output lands in its own buffer.  On the
    forced non-ppw paths the wrapper falls back to one launch per problem (same results)."""
    K_ = _k()
    from dphubert_amd import _lib
    items = [(rnd(M, N), rnd(M, K), torch.randn(N, K, device="cuda")) for _ in range(n)]
    ref = [dy.double().t() @ x.double() + dw.double() for dy, x, dw in items]
    if gemm_path == "ppw":
        import ctypes as C
        s = K_.choose_splits(N, K, M, batch=n)
        ws = torch.empty(max(1, n * s * N * K), device="cuda")
        dy0, x0, dw0 = items[0]
        args = _lib.DphGemmArgs(N, K, M, n, s, 0, 0, K_.dense(dy0), K_.dense(x0), K_.dense(dw0), K_.OUT_F32_ACCUM, 0,
                                1.0, 0.0, 0, None, None, None, 0, None, None, None, None, None, None, 0, 0,
                                ws.data_ptr(), ws.numel() * 4, 0, 0, None)
        grp = _lib.DphGemmGroup()
        grp.n = n
        for i, (dy, x, dw) in enumerate(items):
            grp.a[i], grp.b[i], grp.c[i] = dy.data_ptr(), x.data_ptr(), dw.data_ptr()
        assert "ppw_gemm_kernel" in K_._variant(args)
        rc = _lib.lib().dph_gemm_grouped(C.byref(args), C.byref(grp), _lib.stream_ptr())
        assert rc == 0, _lib.lib().dph_last_error()
    else:
        keep = K_.linear_wgrad_grouped([(dy, x, dw) for dy, x, dw in items], accumulate=True)
        del keep
    torch.cuda.synchronize()
    for (_, _, dw), r in zip(items, ref):
        close(dw, r, 1e-5)


def test_wgrad_grouped_fallback_misaligned(gemm_path):
    """A group whose fp32 outputs are not 16-byte aligned (a bucket view after an odd-sized parameter) falls back
    to per-problem launches where the grouped kernel cannot store them directly; results are the same."""
    K_ = _k()
    if gemm_path != "ppw":
        pytest.skip("ppw path only")
    n, N, K, M = 4, 256, 192, 2000
    flat = torch.randn(n * N * K + 1, device="cuda")
    items = [(rnd(M, N), rnd(M, K), flat[1 + i * N * K:1 + (i + 1) * N * K].view(N, K)) for i in range(n)]
    ref = [dy.double().t() @ x.double() + dw.double() for dy, x, dw in items]
    keep = K_.linear_wgrad_grouped(items, accumulate=True)
    torch.cuda.synchronize()
    del keep
    for (_, _, dw), r in zip(items, ref):
        close(dw, r, 1e-5)


def _wgrad_args(K_, dy, x, dw):
    from dphubert_amd._lib import DphGemmArgs
    M, N = dy.shape
    Kk = x.shape[1]
    s = K_.choose_splits(N, Kk, M)
    return DphGemmArgs(N, Kk, M, 1, s, 0, 0, K_.dense(dy), K_.dense(x), K_.dense(dw), K_.OUT_F32_ACCUM, 0, 1.0, 0.0, 0,
                       None, None, None, 0, None, None, None, None, None, None, 0, 0, None, 4 * s * N * Kk, 0, 0)


@pytest.mark.parametrize("B,Lin,Cc,O,k,s", [(2, 301, 64, 128, 3, 2), (16, 999, 512, 512, 2, 2),
                                             (3, 2001, 512, 512, 3, 2)])
def test_conv_wgrad_ppw(B, Lin, Cc, O, k, s, gemm_path):
    """conv weight gradient with the B operand in the batched row layout (overlapping windows of stride s*C inside
    each utterance): dW[o][j*C + c] = sum_(b,t) dz[b,t,o] x[b, s t + j, c] (components.py:107)."""
    K_ = _k()
    if gemm_path not in ("ppw", "small"):
        pytest.skip("ppw vs the register-staged kernel")
    Lout = (Lin - k) // s + 1
    x = rnd(B, Lin, Cc)
    dz = rnd(B * Lout, O)
    M = B * Lout
    dwp = torch.empty(O, k * Cc, device="cuda")
    A = K_.mat(dz, row_stride=O)
    Bm = K_.mat(x, row_stride=s * Cc, rows_per_batch=Lout, batch_stride=Lin * Cc)
    splits = K_.choose_splits(O, k * Cc, M)
    keep = K_.gemm(A, Bm, K_.dense(dwp), O, k * Cc, M, a_kcontig=False, b_kcontig=False, c_dtype=K_.OUT_F32,
                   splits=splits)
    torch.cuda.synchronize()
    del keep
    win = x.double().unfold(1, k, s)                     # [B][Lout][C][k]
    win = win.permute(0, 1, 3, 2).reshape(M, k * Cc)     # [B*Lout][k*C] (j major)
    ref = dz.double().t() @ win
    close(dwp, ref, 1e-5)


def test_conv_implicit_gemm():
    # channels-last strided conv (k=3, s=2) as a GEMM with a row-address function
    K_ = _k()
    B, Lin, Cc, O, k, s = 2, 101, 64, 96, 3, 2
    Lout = (Lin - k) // s + 1
    x = rnd(B, Lin, Cc)
    w = rnd(O, Cc, k, scale=0.1)
    wp = w.permute(0, 2, 1).contiguous()       # [O][k][C]
    y = torch.empty(B * Lout, O, device="cuda", dtype=torch.float32)
    A = K_.mat(x, row_stride=s * Cc, rows_per_batch=Lout, batch_stride=Lin * Cc)
    K_.gemm(A, K_.dense(wp.view(O, k * Cc)), K_.dense(y), B * Lout, O, k * Cc, a_kcontig=True, b_kcontig=True,
            c_dtype=K_.OUT_F32)
    ref = torch.nn.functional.conv1d(x.float().transpose(1, 2), w.float(), stride=s).transpose(1, 2).reshape(-1, O)
    close(y, ref, 1e-5)


@pytest.mark.parametrize("M,N,K", [(70, 48, 96), (300, 264, 128)])
def test_batched_zdiv(M, N, K):
    # grouped GEMM: z = b*G + g ; B operand depends only on g
    K_ = _k()
    Bt, G = 3, 4
    A = rnd(Bt * G, M, K)
    W = rnd(G, N, K)
    out = torch.empty(Bt, M, G * N, device="cuda")
    K_.gemm(K_.mat(A, K, z_inner=M * K), K_.mat(W, K, z_div=G, z_outer=0, z_inner=N * K),
            K_.mat(out, G * N, z_div=G, z_outer=M * G * N, z_inner=N), M, N, K, a_kcontig=True, b_kcontig=True,
            c_dtype=K_.OUT_F32, batch=Bt * G)
    ref = torch.einsum("bgmk,gnk->bmgn", A.float().view(Bt, G, M, K), W.float()).reshape(Bt, M, G * N)
    close(out, ref, 1e-5)


def test_dropout_epilogue_rate():
    K_ = _k()
    M, N, K = 512, 512, 64
    x, w = rnd(M, K), rnd(N, K)
    y0 = K_.linear_fwd(x, w, out_dtype=torch.float32)
    y1 = K_.linear_fwd(x, w, out_dtype=torch.float32, dropout_p=0.25, seed=123)
    y2 = K_.linear_fwd(x, w, out_dtype=torch.float32, dropout_p=0.25, seed=123)
    assert torch.equal(y1, y2)
    keep = y1 != 0
    rate = 1 - keep.float().mean().item()
    assert abs(rate - 0.25) < 0.01
    close(y1[keep], y0[keep] / 0.75, 1e-5)


def test_perf_ffn_shape():
    K_ = _k()
    M, N, K = 7984, 3072, 768
    x, w = rnd(M, K), rnd(N, K)
    b = torch.randn(N, device="cuda")
    for _ in range(3):
        K_.linear_fwd(x, w, b, act=K_.ACT_GELU)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        K_.linear_fwd(x, w, b, act=K_.ACT_GELU)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    tf = 2 * M * N * K / ms / 1e9
    print(f"\nFFN1 GEMM {M}x{N}x{K}: {ms*1e3:.1f} us, {tf:.0f} TFLOP/s")


@pytest.mark.parametrize("R,C", [(768, 3072), (2304, 768), (40, 136)])
def test_transposed_image_dgrad(R, C):
    """ops.t_image is an exact transpose, and the input-gradient GEMM on it (both operands
    k-contiguous) matches the mn-contiguous form."""
    from dphubert_amd import ops
    K_ = _k()
    img = rnd(R, C)
    wt = ops.t_image(img)
    assert wt is not None and torch.equal(wt, img.t().contiguous())
    assert ops.t_image(img) is wt            # cached on the image
    dy = rnd(520, R)
    a = K_.linear_dgrad(dy, img)
    b = K_.linear_dgrad(dy, img, w_t=wt)
    torch.cuda.synchronize()
    ref = dy.float() @ img.float()
    close(a, ref, 1e-2)
    close(b, ref, 1e-2)


@pytest.mark.parametrize("act", ["none", "gelu_bwd"])
def test_batched_row_output(act):
    """C in a batched row layout (the conv input-gradient phase GEMMs: rows m of utterance m // L land on every
    other row of that utterance, odd phase) with the direct epilogue: GELU' of an aux input in the same layout,
    column mask, column sums of the stored values and of the mask gradient."""
    K_ = _k()
    Bt, L, N, Kd = 3, 333, 192, 256
    Lin = 2 * L + 1
    M = Bt * L
    A, W = rnd(M, Kd), rnd(N, Kd)
    C = torch.zeros(Bt, Lin, N, device="cuda", dtype=torch.bfloat16)
    aux = rnd(Bt, Lin, N)
    cm = (torch.rand(N, device="cuda") > 0.3).float()
    cso, csa = torch.zeros(N, device="cuda"), torch.zeros(N, device="cuda")
    kw = {}
    if act == "gelu_bwd":
        kw = dict(act=K_.ACT_GELU_BWD, aux_in=aux.view(-1)[N:], colmask=cm, colsum_out=cso, colsum_aux=csa)
    K_.gemm(K_.dense(A), K_.dense(W), K_.mat(C, 2 * N, rows_per_batch=L, batch_stride=Lin * N, offset=N), M, N, Kd,
            a_kcontig=True, b_kcontig=True, **kw)
    torch.cuda.synchronize()
    y = (A.float() @ W.float().t()).view(Bt, L, N)
    want = torch.zeros(Bt, Lin, N, device="cuda")
    if act == "gelu_bwd":
        z = aux.float()[:, 1:2 * L:2]
        g = torch.nn.functional.gelu(z)
        dg = torch.autograd.functional.jacobian(lambda t: torch.nn.functional.gelu(t).sum(), z)
        v = y * dg * cm
        want[:, 1:2 * L:2] = v
        close(cso, v.sum((0, 1)), 2e-2)
        close(csa, (y * g).sum((0, 1)), 2e-2)
    else:
        want[:, 1:2 * L:2] = y
    close(C, want, 1e-2)
    assert torch.count_nonzero(C[:, 0:2 * L + 1:2].float()) == 0      # even rows untouched


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_gelu_dgk_pair_matches_recompute(p):
    """The stored-factor GELU pair (forward pre_out = gelu'(pre)*mask*keep/(1-p), backward v = (dy@W2) * that,
    mask gradient = (dy@W2) * f / mask) against the recomputing pair (pre stored, GELU' and the dropout hash
    recomputed in the backward epilogue) on the same inputs and dropout seed."""
    K_ = _k()
    M, D, F = 1000, 256, 392
    x, w1, w2 = rnd(M, D), rnd(F, D, scale=0.1), rnd(D, F, scale=0.1)
    b1 = torch.randn(F, device="cuda") * 0.1
    cm = (torch.rand(F, device="cuda") + 0.2).clamp(max=1.0)
    cm[::7] = 0.0
    u = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
    dgk = torch.empty_like(u)
    f0 = K_.linear_fwd(x, w1, b1, act=K_.ACT_GELU, pre_out=u, colmask=cm, dropout_p=p, seed=77)
    f1 = K_.linear_fwd(x, w1, b1, act=K_.ACT_GELU, pre_out=dgk, colmask=cm, dropout_p=p, seed=77, pre_dgk=True)
    torch.cuda.synchronize()
    # the same dropout pattern and GELU values (other tile paths may round an element differently by one ulp)
    assert torch.equal(f0 == 0, f1 == 0)
    close(f1, f0, 1e-3)
    dy = rnd(M, D)
    w2t = w2.t().contiguous()
    cs0, ca0 = torch.zeros(F, device="cuda"), torch.zeros(F, device="cuda")
    cs1, ca1 = torch.zeros(F, device="cuda"), torch.zeros(F, device="cuda")
    d0 = K_.linear_dgrad(dy, w2, w_t=w2t, act=K_.ACT_GELU_BWD, aux_in=u, colmask=cm, colsum_out=cs0, colsum_aux=ca0,
                         dropout_p=p, seed=77)
    d1 = K_.linear_dgrad(dy, w2, w_t=w2t, act=K_.ACT_GELU_BWD_DGK, aux_in=dgk, residual=f1, colmask=cm,
                         colsum_out=cs1, colsum_aux=ca1)
    torch.cuda.synchronize()
    close(d1, d0, 1e-2)
    close(cs1, cs0, 1e-2)
    live = cm != 0
    close(ca1[live], ca0[live], 2e-2)
    assert torch.count_nonzero(ca1[~live]) == 0


@pytest.mark.parametrize("M,N,K", [(7984, 768, 3072), (7984, 768, 768), (1000, 264, 512)])
def test_pp_b0_prefetch_bitwise(gemm_path, monkeypatch, M, N, K):
    """The B-n0 prefetch schedule of the one-round 128 x 192 ping-pong grids (pp::Cfg::PF) issues the same MFMAs in
    the same order into every accumulator as the plain schedule: bitwise equal outputs (residual epilogue)."""
    if gemm_path != "pp128x192":
        pytest.skip("one tile path is enough")
    K_ = _k()
    A, B, R = rnd(M, K), rnd(N, K, scale=0.05), rnd(M, N)
    outs = []
    for pf in ("1", "0"):
        monkeypatch.setenv("DPH_PP_B0PF", pf)
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        K_.gemm(K_.dense(A), K_.dense(B), K_.dense(C), M, N, K, a_kcontig=True, b_kcontig=True, residual=R)
        torch.cuda.synchronize()
        outs.append(C)
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))
    close(outs[0], A.float() @ B.float().t() + R.float())


@pytest.mark.parametrize("M,N,K,act", [(7984, 2304, 768, "none"), (2000, 2304, 768, "none"), (7984, 3072, 768, "gelu")])
def test_pp_two_blocks_per_cu_bitwise(gemm_path, monkeypatch, M, N, K, act):
    """Multi-round 128 x 192 grids on the two-blocks-per-CU build (pp::Cfg::M2: the QKV forward's default) run the same
    main loop and epilogue as the one-block build: bitwise equal outputs, forced onto either build (DPH_PP_M2)."""
    if gemm_path != "pp128x192":
        pytest.skip("one tile path is enough")
    K_ = _k()
    A, B = rnd(M, K), rnd(N, K, scale=0.05)
    bias = torch.randn(N, device="cuda")
    kw = dict(act=K_.ACT_GELU, bias=bias) if act == "gelu" else dict(bias=bias)
    outs = []
    monkeypatch.setenv("DPH_PP_FORCE", "15")
    for m2 in ("1", "0"):
        monkeypatch.setenv("DPH_PP_M2", m2)
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        K_.gemm(K_.dense(A), K_.dense(B), K_.dense(C), M, N, K, a_kcontig=True, b_kcontig=True, **kw)
        torch.cuda.synchronize()
        outs.append(C)
    assert torch.equal(outs[0].view(torch.int16), outs[1].view(torch.int16))
    ref = A.float() @ B.float().t() + bias
    close(outs[0], torch.nn.functional.gelu(ref) if act == "gelu" else ref)

