"""Precision probe of one attention layer's q / k gradients (build container only: imports the reference through
tools/gen_golden.py, like the fixture generator).

Runs g14's step (12-layer HuBERT-Base, 1 x 10 s) once in fp32, captures the student's layer-L attention input x, its
head mask and the gradient arriving at the attention module's output, then recomputes that layer's backward in fp64
(exact), in fp32, under bf16 emulation, and under numeric models of the HIP kernels, and prints the rel-L2 of
dW_q / dW_k / dW_v against fp64.  With --save, writes the captured inputs to scratch/attn_probe_L.pt (data only) so
tools/attn_probe_gpu.py can run the HIP attention on exactly these inputs.

  PYTHONDONTWRITEBYTECODE=1 python tools/attn_probe.py [--layer 11] [--save]
"""

import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent))
import gen_golden as gg  # noqa: E402

LAYER = int(sys.argv[sys.argv.index("--layer") + 1]) if "--layer" in sys.argv else 11
cap = {}
_orig = gg.seeded_model
_n = [0]


def seeded_model(cfg, seed):
    m, sd = _orig(cfg, seed)
    _n[0] += 1
    if _n[0] == 2:   # run_step builds the teacher first, then the student
        att = m.encoder.transformer.layers[LAYER].attention
        att.register_forward_hook(lambda mod, inp, out: cap.__setitem__("x", inp[0].detach().clone()))
        att.register_full_backward_hook(lambda mod, gi, go: cap.__setitem__("gout", go[0].detach().clone()))
        if att.hard_concrete_for_heads is not None:
            att.hard_concrete_for_heads.register_forward_hook(
                lambda mod, inp, out: cap.__setitem__("hm", out.detach().clone()))
        cap["mod"] = att
    return m, sd


gg.seeded_model = seeded_model
gg.run_step(gg.no_dropout(gg.HUBERT_BASE_CONFIG), gg.no_dropout(gg.HUBERT_BASE_CONFIG), "0.4,8,12", B=1, S=160000,
            units="conv,head,interm", lambdas=(0.0, 0.0), global_step=5000, sens=False)
att = cap["mod"]
x, gout, hm = cap["x"], cap["gout"], cap.get("hm")
H, HD = att.num_heads, att.head_dim
W = {n: getattr(att, n).weight.detach() for n in ("q_proj", "k_proj", "v_proj", "out_proj")}
Bv = {n: getattr(att, n).bias.detach() for n in ("q_proj", "k_proj", "v_proj", "out_proj")}
print(f"layer {LAYER}: x {tuple(x.shape)}, |gout| {gout.norm():.4g}, head mask {hm}")


def bf(t):
    return t.to(torch.bfloat16).to(t.dtype)


class RoundGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, t):
        return t.clone()

    @staticmethod
    def backward(ctx, g):
        return bf(g)


def layer_grads(dtype, emulate=False):
    """The reference attention (components.py:403-430) in ``dtype``; emulate: bf16 operands as Bf16Emulation."""
    r = (lambda t: bf(t)) if emulate else (lambda t: t)  # noqa: E731
    rg = RoundGrad.apply if emulate else (lambda t: t)   # noqa: E731
    ws = {n: W[n].to(dtype).clone().requires_grad_(True) for n in W}
    bs = {n: Bv[n].to(dtype).clone().requires_grad_(True) for n in Bv}
    xx = x.to(dtype)
    Bsz, L, E = xx.shape

    def lin(n, t):
        t = rg(t + (r(t) - t).detach())
        w = ws[n] + (r(ws[n]) - ws[n]).detach()
        y = torch.nn.functional.linear(t, w, bs[n])
        return rg(y + (r(y) - y).detach())

    shape = (Bsz, L, H, HD)
    q = lin("q_proj", xx).view(*shape).transpose(2, 1)
    k = lin("k_proj", xx).view(*shape).permute(0, 2, 3, 1)
    v = lin("v_proj", xx).view(*shape).transpose(2, 1)
    s = (att.scaling * q) @ k
    s = s - s.max(dim=-1, keepdim=True)[0]
    s = rg(s)
    p = torch.softmax(s, dim=-1)
    p = p + (r(p) - p).detach()
    o = p @ v
    if hm is not None:
        o = o * hm.to(dtype).view(1, H, 1, 1)
    o = o.transpose(2, 1).reshape(Bsz, L, H * HD)
    y = lin("out_proj", o)
    y.backward(gout.to(dtype))
    return {n: ws[n].grad.double() for n in ("q_proj", "k_proj", "v_proj")}


def rel(a, b):
    return ((a - b).norm() / b.norm()).item()


exact = layer_grads(torch.float64)
for name, g in (("fp32", layer_grads(torch.float32)), ("bf16-emulated", layer_grads(torch.float32, True))):
    print(name, {n: round(rel(g[n], exact[n]), 4) for n in exact})
if "--save" in sys.argv:
    out = Path(__file__).resolve().parents[1] / "scratch" / f"attn_probe_{LAYER}.pt"
    out.parent.mkdir(exist_ok=True)
    torch.save({"x": x, "gout": gout, "hm": hm, "W": W, "b": Bv, "scaling": att.scaling, "H": H,
                "exact": exact}, out)
    print("saved", out)
