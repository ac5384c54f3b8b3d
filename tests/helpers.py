"""Shared test helpers: rebuild fixture inputs from seeds (no checkpoints shipped)."""

from pathlib import Path

import torch

from dphubert_amd.synthetic import seeded_tensor
from oracle import hubert_ref as ref

GOLDEN = Path(__file__).resolve().parent / "golden"


def load_golden(name):
    return torch.load(GOLDEN / name, map_location="cpu", weights_only=True)


def seeded_sd(cfg, seed):
    return {n: seeded_tensor(n, s, seed) for n, s in ref.state_dict_shapes(cfg)}


def proj_sd_from_recipe(n_proj, D, seed):
    """Distill projection init used by tools/gen_golden.py (identity + seeded delta)."""
    sd = {}
    for g in range(n_proj):
        sd[f"{g}.weight"] = torch.eye(D) + seeded_tensor(f"proj{g}.weight", (D, D), seed) * 0.05
        sd[f"{g}.bias"] = seeded_tensor(f"proj{g}.bias", (D,), seed)
    return sd


def wave_batch(B, S, seed=2022, lengths=None):
    g = torch.Generator()
    g.manual_seed(seed)
    w = 0.1 * torch.randn(B, S, generator=g)
    if lengths is None:
        lengths = [S] * B
    ln = torch.tensor(lengths, dtype=torch.int64)
    for b, l in enumerate(lengths):
        w[b, int(l):] = 0.0
    return w, ln


def rel_l2(a, b):
    a = a.double()
    b = b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def ck_close(t, ck, rtol=1e-5, atol=1e-6):
    """Compare a tensor with a golden checksum dict: (max |sample err| / max |sample|, relative sum-of-squares
    error)."""
    e_max, _, e_sq = ck_errors(t, ck, atol)
    return e_max, e_sq


def ck_errors(t, ck, atol=1e-6):
    """(max |sample err| / max |sample|, rel-L2 of the sampled entries, relative sum-of-squares error)."""
    t = t.detach().double().flatten()
    assert t.numel() == ck["n"], (t.numel(), ck["n"])
    s = t[ck["sample_idx"]]
    want = ck["sample"].double()
    err = (s - want).abs().max().item()
    scale = want.abs().max().item() + atol
    rl2 = ((s - want).norm() / want.norm().clamp_min(1e-30)).item()
    sq = (t * t).sum().item()
    return err / scale, rl2, abs(sq - ck["sq"]) / max(ck["sq"], 1e-30)
