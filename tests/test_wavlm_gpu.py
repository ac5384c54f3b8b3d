"""WavLM gated relative-position attention on the HIP path (components.py:486-659) vs the oracle.

* bucket tables from dph_relpos_table vs the reference's own tables (g8 fixture): bit-exact integers;
* a 1-layer WavLM encoder (post-norm and pre-norm) over T = 299 frames -- 3 query blocks of 128 rows and 5 key
  tiles, so the per-block diagonal histograms of the dQ kernel cover interior, first and last blocks -- padded
  batch, forward + backward vs the fp32 CPU oracle with autograd on identical weights.
  Tolerances (bf16 activations): hidden rel-L2 < 1e-2, parameter-gradient rel-L2 < 3e-2.
"""

import copy

import pytest
import torch

from helpers import load_golden, rel_l2, seeded_sd, wave_batch
from oracle import hubert_ref as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bucket_table(T, nb, md):
    from dphubert_amd._lib import call, stream_ptr
    out = torch.empty(2 * T - 1, dtype=torch.int64, device=DEV)
    call("dph_relpos_table", None, None, None, out.data_ptr(), T, 1, 1, nb, md, stream_ptr())
    torch.cuda.synchronize()
    return out.cpu()


def test_relpos_buckets_match_reference():
    fx = load_golden("g8_wavlm.pt")
    for key, (nb, md, T) in (("bucket_320_800_T1000", (320, 800, 1000)), ("bucket_32_40_T200", (32, 40, 200))):
        got = _bucket_table(T, nb, md)
        # row 0 of the reference table = offsets 0 .. T-1 = diagonals T-1 .. 2T-2
        assert torch.equal(got[T - 1:], fx[key]), key
        want = ref.relative_position_bucket(torch.arange(-(T - 1), T), nb, md)
        assert torch.equal(got, want), key


def _wavlm_cfg(pre_norm, remaining=None):
    from dphubert_amd.synthetic import HUBERT_BASE_CONFIG
    c = copy.deepcopy(HUBERT_BASE_CONFIG)
    del c["encoder_num_heads"], c["encoder_head_dim"]
    c.update(encoder_num_layers=1, encoder_use_attention=[True], encoder_use_feed_forward=[True],
             encoder_ff_interm_features=[3072], encoder_total_num_heads=[12],
             encoder_remaining_heads=[remaining or list(range(12))], encoder_num_buckets=320,
             encoder_max_distance=800, encoder_layer_norm_first=pre_norm, encoder_projection_dropout=0.0,
             encoder_attention_dropout=0.0, encoder_ff_interm_dropout=0.0, encoder_dropout=0.0,
             encoder_layer_drop=0.0)
    return c


def _dz_abs_sum(cfg, sd, wave, ln, R):
    """sum over (b, h, t) of |d loss / d gate-logit| from the oracle (the gate-bias sum's condition)."""
    keep = {}
    orig = ref._linear

    def lin(sd_, p, x):
        y = orig(sd_, p, x)
        if "gru_rel_pos_linear" in p:
            y.retain_grad()
            keep["z"] = y
        return y

    osd = {k: v.clone().requires_grad_(v.is_floating_point()) for k, v in sd.items()}
    ref._linear = lin
    try:
        hs, _ = ref.extract_features(osd, cfg, wave, ln)
    finally:
        ref._linear = orig
    (hs[-1] * R).sum().backward()
    return keep["z"].grad.abs().sum((0, 1, 2)).min().item()


@pytest.mark.parametrize("pre_norm,remaining", [(False, None), (True, [0, 2, 3, 5, 6, 7, 9, 11])])
def test_wavlm_layer_fwd_bwd_vs_oracle(pre_norm, remaining):
    from dphubert_amd.wav2vec2.model import wav2vec2_model
    cfg = _wavlm_cfg(pre_norm, remaining)
    sd = seeded_sd(cfg, 5)
    S = 96000
    wave, ln = wave_batch(2, S, lengths=[S, 70000])
    # oracle (fp32 CPU, autograd)
    osd = {k: v.clone().requires_grad_(v.is_floating_point()) for k, v in sd.items()}
    hs, _ = ref.extract_features(osd, cfg, wave, ln)
    T = hs[-1].shape[1]
    assert T == 299
    g = torch.Generator().manual_seed(3)
    R = torch.randn(hs[-1].shape, generator=g)
    (hs[-1] * R).sum().backward()
    # HIP path
    m = wav2vec2_model(**copy.deepcopy(cfg))
    m.load_state_dict(sd)
    m = m.to(DEV).eval()
    out, _ = m.extract_features(wave.to(DEV), ln.to(DEV))
    (out[-1].float() * R.to(DEV)).sum().backward()
    torch.cuda.synchronize()
    assert rel_l2(out[-1].float().cpu(), hs[-1].detach()) < 1e-2
    p = "encoder.transformer.layers.0.attention."
    names = [p + "rel_attn_embed.weight", p + "gru_rel_pos_linear.weight", p + "gru_rel_pos_const",
             p + "q_proj.weight", p + "k_proj.weight", p + "v_proj.weight",
             "encoder.feature_projection.projection.weight"]
    params = dict(m.named_parameters())
    errs = {n: rel_l2(params[n].grad.cpu(), osd[n].grad) for n in names}
    # the gate-bias gradient is a sum over B*H*T logit gradients with ~1e3x cancellation (sum |dz| ~ 60 vs
    # |sum dz| ~ 0.02-0.3 at this shape): bound its error by the sum's condition, sum_n |dz_n| (recomputed
    # here from the oracle's dz = d(bias) per element), not by its own magnitude
    nb = p + "gru_rel_pos_linear.bias"
    db_err = (params[nb].grad.cpu() - osd[nb].grad).abs().max().item()
    print({k: f"{v:.3g}" for k, v in errs.items()}, f"gate bias max abs err {db_err:.3g}")
    for n, e in errs.items():
        assert e < 3e-2, (n, e)
    assert db_err < 2e-3 * _dz_abs_sum(cfg, sd, wave, ln, R)


def test_pruned_wavlm_forward_vs_reference():
    """The reference's pruned WavLM (ragged remaining heads per layer, ragged FFN widths; fixture g9) forward
    on the HIP path, padded batch: hidden rel-L2 < 1e-2."""
    from dphubert_amd.cli import prune_config
    from dphubert_amd.wav2vec2.model import wav2vec2_model
    fx = load_golden("g9_wavlm_prune.pt")
    m = wav2vec2_model(**copy.deepcopy(fx["cfg"]))
    sd = seeded_sd(fx["cfg"], fx["seed"])
    sd.update(fx["log_alpha"])
    m.load_state_dict(sd)
    pcfg = prune_config(m, fx["cfg"])
    pm = wav2vec2_model(**copy.deepcopy(pcfg))
    pm.load_state_dict(m.state_dict(), strict=True)
    pm = pm.to(DEV).eval()
    with torch.no_grad():
        hs, _ = pm.extract_features(fx["wave"].to(DEV), fx["lengths"].to(DEV))
    torch.cuda.synchronize()
    for h, g in zip(hs, fx["pruned_hiddens"]):
        e = rel_l2(h.float().cpu(), g)
        assert e < 1e-2, e


@pytest.mark.parametrize("T", [3584, 3000])
def test_relpos_backward_long_T_deterministic(T):
    """The relative-position attention backward at its largest supported length (T = 3584: the [T+127] table
    window plus, in deterministic mode, four per-wave diagonal histograms in LDS): deterministic mode runs and
    agrees with the atomic mode (dqkv, dgate, drel_tab rel-L2 <= 1e-4) -- the LDS footprint limit of
    dph_attention_bwd_relpos."""
    import ctypes as C
    from dphubert_amd import _lib
    from dphubert_amd._lib import call, stream_ptr
    B, H = 1, 2
    g = torch.Generator(device="cuda").manual_seed(3)
    qkv = (torch.randn(B * T, 3 * H * 64, device="cuda", generator=g) * 0.5).to(torch.bfloat16)
    tab = torch.randn(H, 2 * T - 1, device="cuda", generator=g) * 0.1
    gate = torch.rand(B, H, T, device="cuda", generator=g)
    o_u = torch.empty(B * T, H * 64, device="cuda")
    o_m = torch.empty(B * T, H * 64, device="cuda", dtype=torch.bfloat16)
    lse = torch.empty(B * H * T, device="cuda")
    ptr = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None  # noqa: E731
    call("dph_attention_fwd_relpos", ptr(qkv), ptr(o_u), ptr(o_m), ptr(lse), None, None, ptr(tab), ptr(gate),
         B, T, H, 0.125, 0.0, 0, None, stream_ptr())
    do = (torch.randn(B * T, H * 64, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
    D = torch.empty(B * H * T, device="cuda")
    dhm = torch.zeros(H, device="cuda")
    pws = torch.empty(max(1, _lib.lib().dph_attention_bwd_prep_workspace(B, T, H) // 4 + 1), device="cuda")
    call("dph_attention_bwd_prep", ptr(do), ptr(o_u), None, ptr(D), ptr(dhm), B, T, H, ptr(pws), pws.numel() * 4,
         stream_ptr())
    res = {}
    prev = _lib.lib().dph_get_deterministic()
    try:
        for det in (1, 0):
            _lib.lib().dph_set_deterministic(det)
            dqkv = torch.empty_like(qkv)
            dgate = torch.empty_like(gate)
            dtab = torch.zeros_like(tab)
            nws = _lib.lib().dph_attention_bwd_relpos_workspace(B, T, H)
            ws = torch.empty(nws // 4 + 1, device="cuda")
            call("dph_attention_bwd_relpos", ptr(qkv), ptr(do), None, ptr(lse), ptr(D), ptr(dqkv), None, ptr(tab),
                 ptr(gate), ptr(dgate), ptr(dtab), B, T, H, 0.125, 0.0, 0, None, ptr(ws), ws.numel() * 4,
                 stream_ptr())
            torch.cuda.synchronize()
            res[det] = (dqkv.float(), dgate, dtab)
    finally:
        _lib.lib().dph_set_deterministic(prev)
    for a, b in zip(res[1], res[0]):
        assert torch.isfinite(a).all()
        assert rel_l2(a.cpu(), b.cpu()) <= 1e-4, rel_l2(a.cpu(), b.cpu())
