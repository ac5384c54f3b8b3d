"""Bitwise A/B of the attention backward across two builds of the library: one forward (dropout 0.1, stored keep
bits) + backward-prep + backward at the distill shape (B = 16, T = 499, H = 12) with head masks in (0.5, 1] and
some utterances padded (key_len < T), seeded; writes dqkv (and D) to OUT.  Run once per build and compare:

    DPH_LIB_PATH=ab/base.so python tools/attn_bitwise.py gpurun_out/a.pt
    python tools/attn_bitwise.py gpurun_out/b.pt --compare gpurun_out/a.pt
"""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
from dphubert_amd import _lib  # noqa: E402
from dphubert_amd._lib import call, ptr  # noqa: E402
from dphubert_amd.ops import _ws  # noqa: E402

out = sys.argv[1]
B, T, H, dev = 16, 499, 12, "cuda"
E = H * 64
g = torch.Generator().manual_seed(7)
qkv = (torch.randn(B * T, 3 * E, generator=g) * 1.5).to(torch.bfloat16).to(dev)
dom = (torch.randn(B * T, E, generator=g) * 0.01).to(torch.bfloat16).to(dev)
hm = (0.5 + 0.5 * torch.rand(H, generator=g)).to(dev)
klen = torch.full((B,), T, dtype=torch.int64)
klen[3], klen[9] = 401, 250
klen = klen.to(dev)
s = _lib.stream_ptr()
res = {}
for label, p, kl in (("drop_keep", 0.1, klen), ("nodrop_full", 0.0, None)):
    o_u = torch.empty(B * T, E, device=dev)
    o_m = torch.empty(B * T, E, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * H * T, device=dev)
    keep = torch.zeros(_lib.lib().dph_attention_keep_bytes(B, T, H), device=dev, dtype=torch.uint8) if p else None
    kp = ptr(kl) if kl is not None else None
    call("dph_attention_fwd", ptr(qkv), ptr(o_u), ptr(o_m), ptr(lse), ptr(hm), kp, B, T, H, 0.125, p, 1234,
         ptr(keep) if keep is not None else None, s)
    Dv = torch.empty(B * H * T, device=dev)
    dhm = torch.zeros(H, device=dev)
    call("dph_attention_bwd_prep", ptr(dom), ptr(o_u), ptr(hm), ptr(Dv), ptr(dhm), B, T, H,
         *_ws(_lib.lib().dph_attention_bwd_prep_workspace(B, T, H), dev), s)
    dqkv = torch.empty_like(qkv)
    call("dph_attention_bwd", ptr(qkv), ptr(dom), ptr(hm), ptr(lse), ptr(Dv), ptr(dqkv), kp, B, T, H, 0.125, p,
         1234, ptr(keep) if keep is not None else None, s)
    torch.cuda.synchronize()
    res[label] = {"dqkv": dqkv.cpu(), "o_m": o_m.cpu(), "D": Dv.cpu()}
torch.save(res, out)
print(f"wrote {out} ({_lib.lib_path() if hasattr(_lib, 'lib_path') else ''})")
if "--compare" in sys.argv:
    ref = torch.load(sys.argv[sys.argv.index("--compare") + 1], weights_only=True)
    ok = True
    for label in res:
        for k in res[label]:
            a, b = res[label][k], ref[label][k]
            same = torch.equal(a.view(torch.int16) if a.dtype == torch.bfloat16 else a,
                               b.view(torch.int16) if b.dtype == torch.bfloat16 else b)
            nd = (a.float() != b.float()).sum().item()
            print(f"{label:12s} {k:5s} bitwise {'equal' if same else 'DIFFERENT'} ({nd} elements differ)")
            ok = ok and same
    sys.exit(0 if ok else 1)
