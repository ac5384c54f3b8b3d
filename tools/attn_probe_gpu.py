"""GPU half of tools/attn_probe.py: the HIP attention forward + backward on one captured layer (scratch/attn_probe_L.pt),
dW_q / dW_k / dW_v formed in fp64 from the kernel's dq / dk / dv, against the fp64 reference gradients; beside it the
fp64 attention on the SAME bf16 q / k / v / dO the kernel read (isolates the kernel's arithmetic from the rounding
of its inputs).

  python tools/attn_probe_gpu.py [--layer 11]
"""

import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
from dphubert_amd import _lib  # noqa: E402
from dphubert_amd._lib import call, ptr  # noqa: E402

LAYER = int(sys.argv[sys.argv.index("--layer") + 1]) if "--layer" in sys.argv else 11
d = torch.load(REPO / "scratch" / f"attn_probe_{LAYER}.pt", weights_only=True)
dev = "cuda"
x = d["x"][0]                      # T x E
T, E = x.shape
H = d["H"]
HD = E // H
B = 1
W, bias = d["W"], d["b"]
hm = d["hm"] if d["hm"] is not None else torch.ones(H)
xb = x.to(torch.bfloat16)
Wqkv = torch.cat([W["q_proj"], W["k_proj"], W["v_proj"]]).to(torch.bfloat16)
bqkv = torch.cat([bias["q_proj"], bias["k_proj"], bias["v_proj"]])
qkv = (xb.float() @ Wqkv.float().t() + bqkv).to(torch.bfloat16)
dom = (d["gout"][0] @ W["out_proj"].to(torch.bfloat16).float()).to(torch.bfloat16)   # grad at out_proj's input

qkv_d, dom_d, hm_d = qkv.to(dev), dom.to(dev), hm.float().to(dev)
o_u = torch.empty(T, E, device=dev)
o_m = torch.empty(T, E, device=dev, dtype=torch.bfloat16)
lse = torch.empty(B * H * T, device=dev)
s = _lib.stream_ptr()
call("dph_attention_fwd", ptr(qkv_d), ptr(o_u), ptr(o_m), ptr(lse), ptr(hm_d), None, B, T, H, float(d["scaling"]),
     0.0, 0, None, s)
Dv = torch.empty(B * H * T, device=dev)
dhm = torch.zeros(H, device=dev)
from dphubert_amd.ops import _ws  # noqa: E402
call("dph_attention_bwd_prep", ptr(dom_d), ptr(o_u), ptr(hm_d), ptr(Dv), ptr(dhm), B, T, H,
     *_ws(_lib.lib().dph_attention_bwd_prep_workspace(B, T, H), dev), s)
dqkv = torch.empty_like(qkv_d)
call("dph_attention_bwd", ptr(qkv_d), ptr(dom_d), ptr(hm_d), ptr(lse), ptr(Dv), ptr(dqkv), None, B, T, H,
     float(d["scaling"]), 0.0, 0, None, s)
torch.cuda.synchronize()
dqkv = dqkv.double().cpu()

# fp64 attention on the kernel's own bf16 inputs
xq = qkv.double().clone().requires_grad_(True)
q, k, v = xq.view(T, 3, H, HD).permute(1, 2, 0, 3)
w = (d["scaling"] * q) @ k.transpose(-1, -2)
p = torch.softmax(w - w.max(-1, keepdim=True)[0], -1)
o = (p @ v) * hm.double().view(H, 1, 1)
o.permute(1, 0, 2).reshape(T, E).backward(dom.double())
g64 = xq.grad

print(f"layer {LAYER}: max P mean {p.max(-1)[0].mean():.4f}, min row max {p.max(-1)[0].min():.4f}")
xd = xb.double()
names = ("q_proj", "k_proj", "v_proj")
for i, n in enumerate(names):
    want = d["exact"][n]
    got = dqkv[:, i * E:(i + 1) * E].t() @ xd
    ref_in = g64[:, i * E:(i + 1) * E].t() @ xd
    rel = lambda a, b: ((a - b).norm() / b.norm()).item()  # noqa: E731
    print(f"{n}: kernel vs fp64-exact {rel(got, want):.4g}; fp64-on-kernel-inputs vs exact {rel(ref_in, want):.4g}; "
          f"kernel vs fp64-on-kernel-inputs {rel(got, ref_in):.4g}; raw d{n[0]} kernel vs fp64-same-inputs "
          f"{rel(dqkv[:, i * E:(i + 1) * E], g64[:, i * E:(i + 1) * E]):.4g}")
