"""The stochastic path the bench times, checked distributionally (SURVEY 7 "Stochasticity"): device-RNG
HardConcrete noise (batched gate launch), attention-probability dropout and LayerNorm-branch dropout.

Parity fixtures run with injected noise / p = 0; these tests pin what the training-mode kernels draw:
  * HardConcrete (hardconcrete.py:96-99): u ~ U(eps, 1 - eps); P(mask > 0) = sigmoid(log_alpha - beta*ln(-l/r))
    (the quantity l0_norm() sums, hardconcrete.py:76-83); E[mask] = the integral over u of the clamped stretched
    sigmoid (fp64 quadrature); fresh noise per RNG epoch, identical noise for identical (seed, epoch);
  * attention dropout (components.py:420 F.dropout on the softmax probabilities): keep rate 1 - p, kept
    probabilities scaled by 1 / (1 - p);
  * residual-branch dropout fused into the LayerNorm (components.py:845 / :273 dropout): same two properties.
"""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
BETA, LO, HI, EPS = 2.0 / 3.0, -0.1, 1.1, 1e-6


def _bank_call(las, u_flat, mask_flat, seed, u_in=None):
    from dphubert_amd import ops
    rows, off = [], 0
    for i, la in enumerate(las):
        rows.append((la.data_ptr(), None if u_in is None else u_in[i].data_ptr(), None, None, la.numel(), off))
        off += la.numel()
    ops.call("dph_hc_bank_fwd", ops._hc_entries(rows), len(rows), ops.ptr(u_flat), ops.ptr(mask_flat), seed, BETA,
             LO, HI, EPS, ops._s())


def _expected_mask(la: torch.Tensor, n: int = 200001) -> torch.Tensor:
    """E[clamp(sigmoid((logit u + la)/beta) * (r - l) + l, 0, 1)], u ~ U(0, 1): midpoint rule in fp64."""
    u = (torch.arange(n, dtype=torch.float64) + 0.5) / n
    lg = torch.log(u) - torch.log1p(-u)
    s = torch.sigmoid((lg[None, :] + la.double().cpu()[:, None]) / BETA)
    return (s * (HI - LO) + LO).clamp(0, 1).mean(1)


def test_hc_bank_matches_per_module_kernel_with_injected_noise():
    from dphubert_amd import ops
    torch.manual_seed(0)
    las = [torch.randn(n, device=DEV) * 2 for n in (512, 12, 3072, 1)]
    us = [torch.rand(la.shape, device=DEV) * 0.98 + 0.01 for la in las]
    tot = sum(la.numel() for la in las)
    u_flat = torch.empty(tot, device=DEV)
    m_flat = torch.empty(tot, device=DEV)
    _bank_call(las, u_flat, m_flat, 7, u_in=us)
    off = 0
    for la, u in zip(las, us):
        m = torch.empty_like(la)
        ops.call("dph_hc_sample_fwd", ops.ptr(la), ops.ptr(u), None, ops.ptr(m), la.numel(), 7, BETA, LO, HI, EPS,
                 ops._s())
        assert torch.equal(m_flat[off:off + la.numel()], m)
        assert torch.equal(u_flat[off:off + la.numel()], u)
        off += la.numel()
    # backward: one launch vs the per-module kernel
    dms = [torch.randn_like(la) for la in las]
    got = [torch.zeros_like(la) for la in las]
    rows, off = [], 0
    for la, dm, g in zip(las, dms, got):
        rows.append((la.data_ptr(), None, dm.data_ptr(), g.data_ptr(), la.numel(), off))
        off += la.numel()
    ops.call("dph_hc_bank_bwd", ops._hc_entries(rows), len(rows), ops.ptr(u_flat), BETA, LO, HI, ops._s())
    for la, u, dm, g in zip(las, us, dms, got):
        want = torch.zeros_like(la)
        ops.call("dph_hc_sample_bwd", ops.ptr(la), ops.ptr(u), ops.ptr(dm), ops.ptr(want), la.numel(), BETA, LO, HI,
                 ops._s())
        torch.testing.assert_close(g, want, rtol=0, atol=0)


def test_hc_bank_more_entries_than_one_launch():
    """> DPH_HC_BANK_CHUNK gates (HuBERT-Large with all five units has 103): chunked launches, same result."""
    from dphubert_amd import ops
    torch.manual_seed(1)
    las = [torch.randn(16 if i % 3 else 1, device=DEV) for i in range(75)]
    us = [torch.rand(la.shape, device=DEV) * 0.98 + 0.01 for la in las]
    tot = sum(la.numel() for la in las)
    u_flat, m_flat = torch.empty(tot, device=DEV), torch.empty(tot, device=DEV)
    _bank_call(las, u_flat, m_flat, 3, u_in=us)
    want = torch.cat([(torch.sigmoid((torch.log(u) - torch.log1p(-u) + la) / BETA) * (HI - LO) + LO).clamp(0, 1)
                      for la, u in zip(las, us)])
    torch.testing.assert_close(m_flat, want, rtol=1e-5, atol=1e-6)


def test_hc_device_rng_distribution():
    from dphubert_amd.stepstate import step_scalars
    step_scalars(torch.device(DEV))                 # the RNG epoch block the kernels read
    la = torch.linspace(-3.0, 3.0, 48, device=DEV)
    las = [la, la.clone(), la.clone()]              # three gates: their noise must be independent
    tot = sum(x.numel() for x in las)
    draws = 3000
    u_all = torch.empty(draws, tot, device=DEV)
    m_all = torch.empty(draws, tot, device=DEV)
    from dphubert_amd.ops import SeedSource
    seeds = SeedSource(1000)          # the per-call 64-bit seeds production draws (splitmix64 of a counter)
    for i in range(draws):
        _bank_call(las, u_all[i], m_all[i], seeds.next())
    u = u_all.double().cpu()
    m = m_all.double().cpu()
    assert u.min().item() >= EPS and u.max().item() <= 1 - EPS
    # uniform: mean 1/2, variance 1/12 (n = 432k draws)
    assert abs(u.mean().item() - 0.5) < 5 * math.sqrt(1 / 12 / u.numel())
    assert abs(u.var().item() - 1 / 12) < 1e-3
    # the three gates (same log_alpha) draw different noise
    assert (u[:, :48] - u[:, 48:96]).abs().mean().item() > 0.2
    # P(mask > 0) = sigmoid(log_alpha + bias) (l0_norm's summand) and E[mask] by quadrature
    bias = -BETA * math.log(-LO / HI)
    p_open = torch.sigmoid(la.double().cpu() + bias)
    for g in range(3):
        mg = m[:, g * 48:(g + 1) * 48]
        emp = (mg > 0).double().mean(0)
        sd = (p_open * (1 - p_open) / draws).sqrt()
        assert ((emp - p_open).abs() <= 5 * sd + 1e-3).all(), (emp - p_open).abs().max()
        em = mg.mean(0)
        want = _expected_mask(la)
        sd_m = mg.std(0) / math.sqrt(draws)
        assert ((em - want).abs() <= 5 * sd_m + 1e-3).all(), (em - want).abs().max()


def test_hc_noise_follows_the_rng_epoch():
    """Graph replays advance the per-step epoch: same seed + new epoch -> new noise; same (seed, epoch) -> the same
    noise (what lets backward kernels regenerate the forward's draws)."""
    from dphubert_amd.stepstate import step_scalars
    blk = step_scalars(torch.device(DEV))
    la = torch.zeros(4096, device=DEV)
    u1, u2, u3 = (torch.empty(4096, device=DEV) for _ in range(3))
    m = torch.empty(4096, device=DEV)
    blk.upload(advance_epoch=True)
    _bank_call([la], u1, m, 42)
    _bank_call([la], u2, m, 42)
    blk.upload(advance_epoch=True)
    _bank_call([la], u3, m, 42)
    torch.cuda.synchronize()
    assert torch.equal(u1, u2)
    assert (u1 - u3).abs().mean().item() > 0.2


def test_model_gates_use_one_launch_and_match_reference_semantics():
    """Student in training mode: every gate comes from the batched launch; masks lie in [0, 1]; backward gives
    the same log_alpha gradients as the per-module path on the same injected noise."""
    import copy
    from dphubert_amd.synthetic import HUBERT_BASE_CONFIG
    from dphubert_amd.trainer import seeded_model, units_flags
    from dphubert_amd.wav2vec2.hardconcrete import HardConcrete
    cfg = copy.deepcopy(HUBERT_BASE_CONFIG)
    cfg.update(encoder_num_layers=1, encoder_use_attention=[True], encoder_use_feed_forward=[True],
               encoder_num_heads=[12], encoder_ff_interm_features=[3072], **units_flags("conv,head,interm,attlayer"))
    m = seeded_model(cfg, 0).to(DEV).train()
    hcs = [x for x in m.modules() if isinstance(x, HardConcrete)]
    g = torch.Generator().manual_seed(5)
    for h in hcs:
        h.set_noise(torch.rand(h.log_alpha.shape, generator=g) * 0.98 + 0.01)
    m._sample_gates()
    assert all(h._bank_mask is not None for h in hcs)
    masks = [h() for h in hcs]
    num = m.get_num_params()
    m._drop_gates()
    w = torch.randn(sum(x.numel() for x in masks), device=DEV)
    loss = torch.cat([x.flatten() for x in masks]).mul(w).sum() + 1e-6 * num
    loss.backward()
    bank_grads = [h.log_alpha.grad.clone() for h in hcs]
    for h in hcs:
        h.log_alpha.grad = None
    # per-module path (no bank) on the same noise
    masks2 = [h() for h in hcs]
    for a, b in zip(masks, masks2):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
        assert a.min().item() >= 0 and a.max().item() <= 1
    num2 = m.get_num_params()
    torch.testing.assert_close(num, num2, rtol=1e-6, atol=0)
    loss2 = torch.cat([x.flatten() for x in masks2]).mul(w).sum() + 1e-6 * num2
    loss2.backward()
    for h, gb in zip(hcs, bank_grads):
        torch.testing.assert_close(gb, h.log_alpha.grad, rtol=1e-5, atol=1e-9)


def test_attention_dropout_keep_rate_and_scale():
    """q = k = 0 -> uniform softmax P = 1/T; V = identity (T = hd = 64) -> O[q, d] = keep(q, d) / (T (1 - p)):
    every output element is one dropout draw of one probability."""
    from dphubert_amd import _lib
    from dphubert_amd._lib import call, ptr
    B, T, H, p = 8, 64, 12, 0.1
    D = H * 64
    qkv = torch.zeros(B, T, 3, H, 64, device=DEV)
    qkv[:, :, 2] = torch.eye(64, device=DEV)[None, :, None, :]
    qkv = qkv.reshape(B * T, 3 * D).to(torch.bfloat16).contiguous()
    hm = torch.ones(H, device=DEV)
    lens = torch.full((B,), T, device=DEV, dtype=torch.int64)
    o_u = torch.empty(B * T, D, device=DEV, dtype=torch.float32)
    o_m = torch.empty(o_u.shape, device=o_u.device, dtype=torch.bfloat16)
    lse = torch.empty(B * H * T, device=DEV)
    call("dph_attention_fwd", ptr(qkv), ptr(o_u), ptr(o_m), ptr(lse), ptr(hm), ptr(lens), B, T, H, 0.125, p, 99, None,
         _lib.stream_ptr())
    o = o_m.float().cpu()
    kept = o != 0
    rate = kept.double().mean().item()
    n = o.numel()
    assert abs(rate - (1 - p)) < 5 * math.sqrt(p * (1 - p) / n), rate
    scale = 1.0 / (T * (1 - p))
    torch.testing.assert_close(o[kept], torch.full_like(o[kept], scale), rtol=8e-3, atol=0)
    # unmasked output (saved for the head-mask gradient) carries the same dropout draws
    assert torch.equal(o_u.float().cpu() != 0, kept)


def test_model_step_passes_stored_keep_bits(monkeypatch):
    """Training step with attention dropout: the forward stores keep bits and the backward reads them (a non-null
    keep pointer on both calls); no-grad forwards pass none."""
    import copy
    from dphubert_amd import ops
    from dphubert_amd.synthetic import HUBERT_BASE_CONFIG
    from dphubert_amd.trainer import seeded_model
    cfg = copy.deepcopy(HUBERT_BASE_CONFIG)
    # (layer drop 0: with HuBERT-Base's 0.05 the single layer is skipped in 1 of 20 steps, depending on the global
    # RNG state the earlier tests of the process left behind)
    cfg.update(encoder_num_layers=1, encoder_attention_dropout=0.1, encoder_layer_drop=0.0)
    m = seeded_model(cfg, 0).to(DEV).train()
    seen = []
    real = ops.call

    def spy(name, *args):
        # (keep_bits: argument 12 of the forward, 13 of the backward -- dph_attention_bwd_qv, ABI 24, appends the
        # q / v bias outputs after it)
        if name == "dph_attention_fwd":
            seen.append((name, args[12]))
        elif name in ("dph_attention_bwd", "dph_attention_bwd_qv"):
            seen.append(("dph_attention_bwd", args[13]))
        return real(name, *args)
    monkeypatch.setattr(ops, "call", spy)
    wave = torch.randn(2, 16000, device=DEV) * 0.1
    x, _ = m(wave)
    x.float().pow(2).mean().backward()
    torch.cuda.synchronize()
    assert [n for n, _ in seen] == ["dph_attention_fwd", "dph_attention_bwd"], seen
    assert all(k not in (None, 0) for _, k in seen), seen
    assert seen[0][1] == seen[1][1]
    seen.clear()
    with torch.no_grad():
        m(wave)
    # (a no-grad forward stores no keep bits, whichever attention entry it goes through)
    assert all(k in (None, 0) for _, k in seen), seen


def test_layernorm_branch_dropout_keep_rate_and_scale():
    from dphubert_amd import _lib
    from dphubert_amd._lib import call, ptr
    torch.manual_seed(3)
    rows, D, p = 4096, 768, 0.1
    x = torch.randn(rows, D, device=DEV).to(torch.bfloat16)
    gamma = torch.rand(D, device=DEV) + 0.5
    beta = torch.randn(D, device=DEV) * 0.1
    y = torch.empty(rows, D, device=DEV, dtype=torch.bfloat16)
    mean = torch.empty(rows, device=DEV)
    rstd = torch.empty(rows, device=DEV)
    call("dph_layernorm_fwd", ptr(x), None, ptr(gamma), ptr(beta), ptr(y), ptr(mean), ptr(rstd), rows, D, 1e-5, p,
         1234, _lib.stream_ptr())
    ref = torch.nn.functional.layer_norm(x.float(), (D,), gamma, beta, 1e-5)
    yf = y.float()
    kept = yf != 0
    rate = kept.double().mean().item()
    assert abs(rate - (1 - p)) < 5 * math.sqrt(p * (1 - p) / yf.numel()) + 1e-4, rate
    r = ref[kept] / (1 - p)
    assert ((yf[kept] - r).abs() <= 1e-2 * r.abs() + 2e-2).all()
    # p = 0: no element dropped
    call("dph_layernorm_fwd", ptr(x), None, ptr(gamma), ptr(beta), ptr(y), ptr(mean), ptr(rstd), rows, D, 1e-5, 0.0,
         1234, _lib.stream_ptr())
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=2e-2)
