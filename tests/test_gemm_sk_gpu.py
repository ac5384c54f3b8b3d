"""The persistent stream-K ping-pong GEMM (gemm_sk.hip: 256 x 256 tiles, K-tile ranges cut across blocks, fp32 tail
pieces handed to the tile's owner by write-through stores + an agent-scope flag) against a torch fp32 reference of the
same op, against the tile kernels, and run to run (the owner adds the partial in a fixed order: bitwise repeatable).
The shapes are the wide-N M = B*T projections it is routed to (QKV forward N = 2304, FFN1 forward / FFN2 input
gradient N = 3072, K = 768) plus ragged M / N / K edges."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _k():
    from dphubert_amd import kernels as K
    return K


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return (torch.randn(*shape, device="cuda", generator=g) * scale).to(torch.bfloat16)


def rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / b.norm().clamp_min(1e-20))


def _plan(M, N, K):
    import ctypes as C
    from dphubert_amd import _lib
    K_ = _k()
    A, B, Cm = rnd(M, K), rnd(N, K), torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    args = _lib.DphGemmArgs(M, N, K, 1, 1, 1, 1, K_.dense(A), K_.dense(B), K_.dense(Cm), K_.OUT_BF16, K_.ACT_NONE, 1.0)
    nb, nf = C.c_int64(0), C.c_int64(0)
    return _lib.lib().dph_gemm_sk_plan(C.byref(args), C.byref(nb), C.byref(nf)), nb.value, nf.value


@pytest.fixture(autouse=True)
def _sk(monkeypatch):
    monkeypatch.delenv("DPH_GEMM_PATH", raising=False)
    monkeypatch.setenv("DPH_GEMM_SK", "1")


def test_routing():
    """Routed: the wide-N projections; not routed: N = 768 (few 256-wide tiles), K not a multiple of 128."""
    assert _plan(7984, 2304, 768)[0] == 1
    assert _plan(7984, 3072, 768)[0] == 1
    ok, nb, nf = _plan(7984, 3072, 768)
    assert nb == 256 * 256 * 256 * 4 and nf == 257          # 256 blocks (one per CU), one slot + flag each
    assert _plan(7984, 768, 3072)[0] == 0
    assert _plan(7984, 2304, 704)[0] == 0


@pytest.mark.parametrize("M,N,K", [(7984, 2304, 768), (7984, 3072, 768), (5988, 4096, 1024), (2000, 2304, 1024),
                                   (7984, 2112, 512), (1000, 3072, 768)])
def test_stream_k_matches_fp32(M, N, K):
    K_ = _k()
    A, B, R = rnd(M, K, seed=1), rnd(N, K, scale=0.05, seed=2), rnd(M, N, seed=3)
    ok = _plan(M, N, K)[0]
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    K_.gemm(K_.dense(A), K_.dense(B), K_.dense(C), M, N, K, a_kcontig=True, b_kcontig=True, residual=R)
    torch.cuda.synchronize()
    ref = A.float() @ B.float().t() + R.float()
    assert rel(C, ref) < 4e-3, (ok, rel(C, ref))
    # bitwise run to run (fixed hand-off order, no atomics on data)
    C2 = torch.empty_like(C)
    K_.gemm(K_.dense(A), K_.dense(B), K_.dense(C2), M, N, K, a_kcontig=True, b_kcontig=True, residual=R)
    torch.cuda.synchronize()
    assert torch.equal(C.view(torch.int16), C2.view(torch.int16))


def test_stream_k_gelu_bias_mask_against_tile_kernel(monkeypatch):
    """FFN1 forward epilogue (bias, exact GELU, column mask) on the stream-K grid against the 128 x 128 ping-pong tile:
    the same math in another K order, so equal to within bf16 rounding of the output."""
    K_ = _k()
    M, N, K = 7984, 3072, 768
    x, w = rnd(M, K, seed=4), rnd(N, K, scale=0.05, seed=5)
    b = torch.randn(N, device="cuda")
    cm = torch.rand(N, device="cuda")
    ys = []
    for sk in ("1", "0"):
        monkeypatch.setenv("DPH_GEMM_SK", sk)
        ys.append(K_.linear_fwd(x, w, b, act=K_.ACT_GELU, colmask=cm))
    torch.cuda.synchronize()
    u = x.float() @ w.float().t() + b
    ref = torch.nn.functional.gelu(u) * cm
    assert rel(ys[0], ref) < 4e-3
    assert rel(ys[0], ys[1]) < 4e-3


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_stream_k_heavy_epilogues(monkeypatch, p):
    """DPH_GEMM_SK=all: the stored-factor GELU pair (forward with dropout and the GELU' factor, the DGK input
    gradient with its column sums) on the stream-K grid equals the tile kernels' results to bf16 rounding."""
    K_ = _k()
    M, N, K = 7984, 3072, 768
    x, w1 = rnd(M, K, seed=6), rnd(N, K, scale=0.05, seed=7)
    w2t = rnd(N, K, scale=0.05, seed=8)        # the FFN2 weight as the (k-contiguous) B of the input gradient
    dy = rnd(M, K, seed=9)
    b1 = torch.randn(N, device="cuda")
    cm = torch.rand(N, device="cuda") + 0.5
    res = {}
    for sk in ("all", "0"):
        monkeypatch.setenv("DPH_GEMM_SK", sk)
        dgk = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        f = K_.linear_fwd(x, w1, b1, act=K_.ACT_GELU, pre_out=dgk, colmask=cm, dropout_p=p, seed=77, pre_dgk=True)
        db = torch.zeros(N, device="cuda")
        dh = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        K_.gemm(K_.dense(dy), K_.dense(w2t), K_.dense(dh), M, N, K, a_kcontig=True, b_kcontig=True,
                act=K_.ACT_GELU_BWD_DGK, aux_in=dgk, colsum_out=db)
        torch.cuda.synchronize()
        res[sk] = (f, dgk, dh, db)
    for a, b in zip(res["all"], res["0"]):
        assert rel(a, b) < 4e-3, rel(a, b)
