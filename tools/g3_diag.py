"""Diagnostic (GPU box): where does the HIP step's gradient leave the fp32 oracle on the 12-layer fixture g3?

Runs the HIP distill step on tests/golden/g3_base12.pt and the fp32 oracle (oracle/hubert_ref.py, plain torch)
on the same device, then prints per-hidden-state gradient rel-L2 and the HardConcrete logit gradients.
"""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from helpers import load_golden, proj_sd_from_recipe, rel_l2, seeded_sd, wave_batch  # noqa: E402
from oracle import hubert_ref as ref  # noqa: E402
from test_parity_gpu import build_module  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "g3_base12.pt"
fx = load_golden(name)
dm = build_module(fx)
wave, ln = wave_batch(fx["B"], fx["S"], lengths=None if fx["lengths"] is None else fx["lengths"].tolist())
cap = {}
orig = dm.student_model.extract_features


def ef(*a, **k):
    r = orig(*a, **k)
    cap["h"] = r[0]
    cap["g"] = [None] * len(r[0])
    for i, h in enumerate(r[0]):
        if h.requires_grad:
            h.register_hook(lambda g, i=i: cap["g"].__setitem__(i, g.detach().float().cpu()))
    return r


dm.student_model.extract_features = ef
loss = dm._step((wave.cuda(), ln.cuda() if fx["lengths"] is not None else None), 0, "train")
loss.backward()
torch.cuda.synchronize()
print("HIP loss", loss.item(), "ref", fx["loss"].item())

# fp32 oracle on the GPU (plain torch ops)
dev = "cuda"
tsd = {k: v.to(dev) for k, v in seeded_sd(fx["tcfg"], fx["seed"]).items()}
ssd = {k: v.to(dev) for k, v in seeded_sd(fx["scfg"], fx["seed"]).items()}
psd = {k: v.to(dev) for k, v in proj_sd_from_recipe(max(fx["proj_index"]) + 1, 768, fx["seed"]).items()}
ocap = {}
o_ef = ref.extract_features


def ef2(sd, cfg, w, lengths=None, masks=None, **k):
    h, l = o_ef(sd, cfg, w, lengths, masks, **k)
    if masks is not None:
        for x in h:
            x.retain_grad()
        ocap["h"] = h
    return h, l


ref.extract_features = ef2
torch.backends.cuda.matmul.allow_tf32 = False
out = ref.distill_step(tsd, fx["tcfg"], ssd, fx["scfg"], psd, fx["distill_layers"], fx["proj_index"], wave.to(dev),
                       None, {k: v.to(dev) for k, v in fx["u"].items()}, fx["lambdas"], fx["global_step"],
                       original_num_params=fx["original_num_params"])
print("oracle(cuda fp32) loss", out["loss"].item())
for i, (g, x) in enumerate(zip(cap["g"], ocap["h"])):
    if g is None or x.grad is None:
        print(f"hidden {i}: grad None (hip {g is None}, oracle {x.grad is None})")
        continue
    print(f"hidden {i}: grad rel-L2 {rel_l2(g, x.grad.float().cpu()):.4g}  |g| {x.grad.norm().item():.4g}")
sdict = dict(dm.student_model.named_parameters())
for n, g in fx["log_alpha_grads"].items():
    got = sdict[n].grad.cpu()
    og = out["grads"][n].float().cpu()
    print(f"{n}: hip-vs-ref {rel_l2(got, g):.4g}  oracle-vs-ref {rel_l2(og, g):.4g}  hip-vs-oracle {rel_l2(got, og):.4g}")
    if rel_l2(got, g) > 0.05:
        print("   hip   ", got[:12].tolist())
        print("   oracle", og[:12].tolist())
        print("   ref   ", g[:12].tolist())

# isolate the loss + projection backward: fp64 torch on the HIP path's own (bf16) student / teacher hiddens
with torch.no_grad():
    th, _ = dm.teacher_model.extract_features(wave.cuda(), None)
hs = [cap["h"][i].detach().double().requires_grad_(True) for i in fx["distill_layers"]]
tt = torch.stack([th[i].double() for i in fx["distill_layers"]], dim=1)
ss = torch.stack([torch.nn.functional.linear(h, dm.distill_linear_projs[j].weight.double(),
                                             dm.distill_linear_projs[j].bias.double()) for j, h in enumerate(hs)], 1)
l64, _ = ref.distill_loss(ss, tt, fx["l2"], 1.0, 1.0, fx["cos_type"])
l64.backward()
for j, i in enumerate(fx["distill_layers"]):
    print(f"loss+proj backward on HIP hiddens, hidden {i}: HIP vs fp64 rel-L2 {rel_l2(cap['g'][i], hs[j].grad.float().cpu()):.4g}")
# and the fp32 oracle's gradient on the oracle's own hiddens vs fp64 on HIP hiddens (forward-difference effect)
for j, i in enumerate(fx["distill_layers"]):
    if i == len(cap["h"]) - 1:
        print(f"hidden {i}: oracle grad vs fp64-on-HIP-hiddens {rel_l2(ocap['h'][i].grad.float().cpu(), hs[j].grad.float().cpu()):.4g}")
d = (ss - tt).abs()
print("fraction |s-t| < 1e-2*|t| (L1 sign-sensitive):", (d < 1e-2 * tt.abs()).double().mean().item())
