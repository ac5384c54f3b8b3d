"""Ping-pong tile A/B on the step's projection GEMMs WITH their epilogues (GELU + stored factor + dropout, fp32
residual stream, DGK input gradient): every tile kind forced through DPH_PP_FORCE (read per call), interleaved
rounds, median us per (shape, tile).  usage: python tools/pp_tile_ab.py [rounds] [kind ...]
kinds: 12 = 256x256, 13 = 128x256, 14 = 256x128, 15 = 128x192, 16 = 128x128 (two blocks per CU).
DPH_AB_SET=conv: the conv extractor's input-gradient GEMMs with the previous layer's GELU backward in the epilogue
(ops.conv_dgrad_phases: M = B x L rows, N = Cin = 512, K = 512 / 1024) instead of the encoder projections."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dphubert_amd import kernels as K  # noqa: E402

M = 16 * 499
dev = "cuda"
bf = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731


def case(name, n, k, m=M, **epi):
    return name, n, k, m, epi


u = torch.empty(M, 3072, device=dev, dtype=torch.bfloat16)
cm = torch.rand(3072, device=dev) + 0.5
res32 = torch.randn(M, 768, device=dev)
MC = 16 * 7999
zc = torch.empty(MC, 512, device=dev, dtype=torch.bfloat16)
cmc = torch.rand(512, device=dev) + 0.5
dmc = torch.zeros(512, device=dev)
CONV = [
    case("conv2 dgrad k=3 odd rows (gelu bwd)", 512, 512, m=MC, act=K.ACT_GELU_BWD, aux_in=zc, colmask=cmc,
         colsum_aux=dmc),
    case("conv3 dgrad k=3 odd rows (gelu bwd)", 512, 512, m=16 * 3999, act=K.ACT_GELU_BWD, aux_in=zc, colmask=cmc,
         colsum_aux=dmc),
    case("conv2 dgrad k=3 even rows (gelu bwd)", 512, 1024, m=MC, act=K.ACT_GELU_BWD, aux_in=zc, colmask=cmc,
         colsum_aux=dmc),
    case("conv1 dgrad k=3 odd rows (no epilogue)", 512, 512, m=16 * 15999),
]
CASES = [
    case("ffn1 fwd student (gelu, gelu' factor, mask, dropout)", 3072, 768, act=K.ACT_GELU, pre_out=u, colmask=cm,
         dropout_p=0.1, seed=3, flags=K.GEMM_PRE_DGK, bias=True),
    case("ffn1 fwd teacher (gelu, pre)", 3072, 768, act=K.ACT_GELU, pre_out=u, bias=True),
    case("ffn2 dgrad DGK", 3072, 768, act=K.ACT_GELU_BWD_DGK, aux_in=u),
    case("qkv fwd", 2304, 768, bias=True),
    case("ffn2 fwd (fp32 residual)", 768, 3072, residual=res32, c_dtype=K.OUT_F32, bias=True),
    case("oproj fwd (fp32 residual)", 768, 768, residual=res32, c_dtype=K.OUT_F32, bias=True),
    case("oproj fwd (bf16 residual, post-norm)", 768, 768, residual=torch.empty(M, 768, device=dev,
                                                                                dtype=torch.bfloat16), bias=True),
    case("ffn2 fwd (bf16 residual, post-norm)", 768, 3072, residual=torch.empty(M, 768, device=dev,
                                                                                dtype=torch.bfloat16), bias=True),
    case("ffn1 dgrad", 768, 3072),
    case("qkv dgrad", 768, 2304),
]
# conv extractor forward (implicit GEMM over overlapping row windows, GELU + stored pre-activation: ops.FrontendFn)
CONVF = []
for li, (lin, lout, kk, st) in enumerate([(31999, 15999, 3, 2), (15999, 7999, 3, 2), (7999, 3999, 3, 2)], start=1):
    xin = bf(16 * lin, 512)
    CONVF.append((f"conv{li} fwd k={kk} (gelu, pre)", 512, kk * 512, 16 * lout,
                  dict(act=K.ACT_GELU, pre=True, win=(xin, st * 512, lout, lin * 512))))
if os.environ.get("DPH_AB_SET") == "conv":
    CASES = CONV
elif os.environ.get("DPH_AB_SET") == "convf":
    CASES = CONVF
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
kinds = sys.argv[2:] or ["auto", "sk0", "skall", "15", "16", "12"]
data = {}
for name, n, k, m, epi in CASES:
    win = epi.pop("win", None)
    if epi.pop("pre", False):
        epi["pre_out"] = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    A, B = (win if win is not None else bf(m, k)), bf(n, k)
    odt = torch.float32 if epi.get("c_dtype") == K.OUT_F32 else torch.bfloat16
    C = torch.empty(m, n, device=dev, dtype=odt)
    kw = dict(epi)
    if kw.pop("bias", False):
        kw["bias"] = torch.randn(n, device=dev)
    data[name] = (A, B, C, m, n, k, kw)


GRAPHS = {}


def run(name, kind, iters=20):
    """kind: "auto" (the library's routing), "sk0" / "skall" (DPH_GEMM_SK=0 / =all, tiles by the library's pick), or
    a ping-pong tile id forced with the stream-K route off.  The iters launches are captured once into a HIP graph
    and replayed (host launch cost out of the measurement)."""
    from dphubert_amd import ops
    os.environ.pop("DPH_PP_FORCE", None)
    os.environ.pop("DPH_GEMM_SK", None)
    os.environ.pop("DPH_PP_M2", None)
    if kind == "m2":          # the 128 x 192 tile on its two-blocks-per-CU build (Cfg::M2)
        os.environ["DPH_PP_M2"] = "1"
        os.environ["DPH_PP_FORCE"] = "15"
    elif kind == "sk0":
        os.environ["DPH_GEMM_SK"] = "0"
    elif kind == "skall":
        os.environ["DPH_GEMM_SK"] = "all"
    elif kind != "auto":
        os.environ["DPH_PP_FORCE"] = kind
        os.environ["DPH_GEMM_SK"] = "0"
    A, B, C, m, n, k, kw = data[name]
    Am = (K.mat(A[0], row_stride=A[1], rows_per_batch=A[2], batch_stride=A[3]) if isinstance(A, tuple)
          else K.dense(A))
    f = lambda: K.gemm(Am, K.dense(B), K.dense(C), m, n, k, a_kcontig=True, b_kcontig=True, **kw)  # noqa
    g = GRAPHS.get((name, kind))
    if g is None:
        f()
        torch.cuda.synchronize()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        ops.reset_zero_arena()
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                f()
        ops.reset_zero_arena()
        GRAPHS[(name, kind)] = g
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


res = {}
for _ in range(rounds):
    for name, *_r in CASES:
        for kd in kinds:
            res.setdefault((name, kd), []).append(run(name, kd))
os.environ.pop("DPH_PP_FORCE", None)
os.environ.pop("DPH_GEMM_SK", None)
os.environ.pop("DPH_PP_M2", None)
for name, n, k, m, _e in CASES:
    fl = 2.0 * m * n * k
    row = " | ".join(f"{kd} {statistics.median(res[(name, kd)]):6.1f}" for kd in kinds)
    best = min(kinds, key=lambda kd: statistics.median(res[(name, kd)]))
    print(f"{name:52s} {m}x{n}x{k}: {row}  (best {best}: "
          f"{fl / statistics.median(res[(name, best)]) / 1e6:5.0f} TF/s)", flush=True)
