"""Pin the CPU oracle (oracle/hubert_ref.py) against golden vectors produced by
importing the reference itself (tools/gen_golden.py).  CPU only."""

import math

import pytest
import torch

from helpers import ck_close, load_golden, proj_sd_from_recipe, rel_l2, seeded_sd, wave_batch
from oracle import hubert_ref as ref


@pytest.fixture(scope="module")
def g1():
    return load_golden("g1_ops.pt")


@pytest.mark.parametrize("key", ["hc_12", "hc_64", "hc_1"])
def test_hardconcrete(g1, key):
    d = g1[key]
    m = ref.hc_sample(d["log_alpha"], d["u"])
    torch.testing.assert_close(m, d["mask"], rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(ref.hc_l0_norm(d["log_alpha"]), d["l0"], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(ref.hc_eval_mask(d["log_alpha"]), d["eval_mask"], rtol=1e-6, atol=1e-7)


def test_distill_loss(g1):
    keys = [k for k in g1 if k.startswith("loss_")]
    assert len(keys) == 4
    for k in keys:
        d = g1[k]
        cos_type = k.split("_")[1] if not k.startswith("loss_log_sig") else "log_sig"
        w = d["w"].tolist()
        s = d["s"].clone().requires_grad_(True)
        loss, (mse, l1, cos) = ref.distill_loss(s, d["t"], w[0], w[1], w[2], cos_type)
        loss.backward()
        torch.testing.assert_close(loss.detach(), d["loss"], rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(l1.detach(), d["l1"], rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(cos.detach(), d["cos"], rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(s.grad, d["grad"], rtol=1e-5, atol=1e-7)


def test_num_params(g1):
    d = g1["num_params"]
    sd = seeded_sd(d["cfg"], d["seed"])
    v = ref.get_num_params(sd, d["cfg"])
    assert abs(float(v) - float(d["value"])) <= 1e-6 * float(d["value"])
    base = {k: v for k, v in d["cfg"].items()}
    for f in ("extractor_prune_conv_channels", "encoder_prune_attention_heads", "encoder_prune_attention_layer",
              "encoder_prune_feed_forward_intermediate", "encoder_prune_feed_forward_layer"):
        base[f] = False
    assert sum(math.prod(s) for _, s in ref.state_dict_shapes(base)) == d["teacher_numel"]


def test_lr_schedule_formula():
    # lightning.py:37-44 restated; spot values
    assert ref.linear_decay_lr(1, 2e-4, 15000, 50000) == pytest.approx(2e-4 / 15000)
    assert ref.linear_decay_lr(15000, 2e-4, 15000, 50000) == pytest.approx(2e-4)
    assert ref.linear_decay_lr(32500, 2e-4, 15000, 50000) == pytest.approx(1e-4)
    assert ref.linear_decay_lr(50000, 2e-4, 15000, 50000) == 0.0


def _run_fixture(fx):
    tcfg, scfg, seed = fx["tcfg"], fx["scfg"], fx["seed"]
    tsd = seeded_sd(tcfg, seed)
    ssd = seeded_sd(scfg, seed)
    n_proj = max(fx["proj_index"]) + 1
    psd = proj_sd_from_recipe(n_proj, scfg["encoder_embed_dim"], seed)
    lengths = fx["lengths"]
    wave, ln = wave_batch(fx["B"], fx["S"], lengths=None if lengths is None else lengths.tolist())
    out = ref.distill_step(tsd, tcfg, ssd, scfg, psd, fx["distill_layers"], fx["proj_index"], wave,
                           ln if lengths is not None else None, fx["u"], fx["lambdas"], fx["global_step"],
                           l2_weight=fx["l2"], cos_type=fx["cos_type"],
                           original_num_params=fx["original_num_params"],
                           distill_mode=fx.get("distill_mode", "layer2layer"))
    return out


def _check_step(fx, out, tol_loss=1e-5, tol_ck=1e-4):
    assert abs(out["loss"].item() - fx["loss"].item()) <= tol_loss * max(1.0, abs(fx["loss"].item()))
    lg = fx["logged"]
    assert abs(out["loss_distill"].item() - lg["train_loss_distill"].item()) <= tol_loss
    assert abs(out["loss_l1"].item() - lg["train_loss_l1"].item()) <= tol_loss
    assert abs(out["loss_cos"].item() - lg["train_loss_cos"].item()) <= tol_loss
    if fx["lambdas"] is not None:
        assert abs(out["expected_sparsity"].item() - lg["sparsity_expected"].item()) <= 1e-6
        assert abs(out["target_sparsity"] - float(lg["sparsity_target"])) <= 1e-7
        for a, b in zip(out["lambda_grads"], fx["lambda_grads"]):
            assert abs(a.item() - b.item()) <= 1e-6 + 1e-5 * abs(b.item())
    for h, ck in zip(out["student_hiddens"], fx["student_hidden_ck"]):
        e_sample, e_sq = ck_close(h, ck)
        assert e_sample < tol_ck and e_sq < tol_ck, (e_sample, e_sq)
    for h, ck in zip(out["teacher_hiddens"], fx["teacher_hidden_ck"]):
        e_sample, e_sq = ck_close(h, ck)
        assert e_sample < tol_ck and e_sq < tol_ck, (e_sample, e_sq)
    for n, g in fx["log_alpha_grads"].items():
        assert rel_l2(out["grads"][n], g) < 1e-3, n
    for n, ck in fx["grad_ck"].items():
        if n.endswith("k_proj.bias"):
            # softmax is shift-invariant per query row, so d/dk_bias is exactly 0;
            # both sides hold only rounding noise (~1e-9), nothing to compare.
            assert out["grads"][n].abs().max().item() < 1e-5
            continue
        e_sample, e_sq = ck_close(out["grads"][n], ck)
        assert e_sq < 1e-3, (n, e_sq)


def test_smoke_step_g2():
    fx = load_golden("g2_smoke_step.pt")
    out = _run_fixture(fx)
    _check_step(fx, out)
    for h, g in zip(out["student_hiddens"], fx["student_hiddens"]):
        assert rel_l2(h, g) < 1e-5


def test_all_units_padded_g2b():
    fx = load_golden("g2b_all_units_padded.pt")
    out = _run_fixture(fx)
    _check_step(fx, out)


@pytest.mark.slow
def test_base12_g3():
    fx = load_golden("g3_base12.pt")
    out = _run_fixture(fx)
    _check_step(fx, out, tol_loss=2e-5, tol_ck=5e-4)


def test_large_whole_g15():
    """g15 (4 pre-norm Large layers, T = 781): the oracle's WHOLE gradients of the stored tensors against the
    reference's (stored in bf16: rel-L2 <= 1e-2 covers their rounding), loss terms and checksums as every step."""
    fx = load_golden("g15_large4_whole.pt")
    out = _run_fixture(fx)
    _check_step(fx, out, tol_loss=2e-5, tol_ck=5e-4)
    assert len(fx["whole_grads"]) >= 20
    for n, w in fx["whole_grads"].items():
        if n.endswith("k_proj.bias"):
            continue
        g = out["grads"][n]
        assert rel_l2(g, w.float()) < 1e-2, (n, rel_l2(g, w.float()))
        assert abs(g.double().norm().item() - fx["whole_norms"][n]) <= 1e-4 * fx["whole_norms"][n], n


def test_oracle_pruned_forward_matches_reference():
    """The oracle restatement on the reference's pruned architecture (ragged widths) -- g4."""
    import copy as _copy
    from dphubert_amd.cli import prune_config
    from dphubert_amd.wav2vec2.model import wav2vec2_model
    from helpers import ck_close, seeded_sd
    fx = load_golden("g4_prune.pt")
    m = wav2vec2_model(**_copy.deepcopy(fx["cfg"]))
    sd = seeded_sd(fx["cfg"], fx["seed"])
    sd.update(fx["log_alpha"])
    m.load_state_dict(sd)
    pcfg = prune_config(m, fx["cfg"])
    psd = {k: v.detach() for k, v in m.state_dict().items()}
    with torch.no_grad():
        hs, _ = ref.extract_features(psd, pcfg, fx["wave"])
    for h, ck in zip(hs, fx["pruned_hidden_ck"]):
        e_sample, e_sq = ck_close(h, ck)
        assert e_sample < 1e-4 and e_sq < 1e-5, (e_sample, e_sq)


def test_prenorm_normalize_waveform_g6():
    """wav2vec2-Large-style layers: pre-norm encoder + per-utterance waveform LayerNorm."""
    fx = load_golden("g6_prenorm_normwave.pt")
    out = _run_fixture(fx)
    _check_step(fx, out)
    for h, g in zip(out["student_hiddens"], fx["student_hiddens"]):
        assert rel_l2(h, g) < 1e-5


def test_layer_norm_extractor_g7():
    """layer_norm-mode extractor with conv bias (LayerNorm over channels after every conv) + pre-norm
    layers: the oracle restatement against the reference's own step on the same inputs."""
    fx = load_golden("g7_lnext.pt")
    out = _run_fixture(fx)
    _check_step(fx, out)
    for h, g in zip(out["student_hiddens"], fx["student_hiddens"]):
        assert rel_l2(h, g) < 1e-5


def test_wavlm_g8():
    """WavLM layers (bucketed relative-position bias shared from layer 0, per-layer gate, a layer with 9 of 12
    heads remaining): the oracle restatement against the reference's own step on the same inputs."""
    fx = load_golden("g8_wavlm.pt")
    assert [(k, tuple(s)) for k, s in ref.state_dict_shapes(fx["scfg"])] == [(k, tuple(s)) for k, s in
                                                                              fx["sd_schema"]]
    out = _run_fixture(fx)
    _check_step(fx, out)
    for h, g in zip(out["student_hiddens"], fx["student_hiddens"]):
        assert rel_l2(h, g) < 1e-5


def test_wavlm_relative_position_bucket():
    """Bucket index tables (integer, bit-exact) for WavLM Base (320 buckets / 800) and a small config."""
    fx = load_golden("g8_wavlm.pt")
    for key, (nb, md, T) in (("bucket_320_800_T1000", (320, 800, 1000)), ("bucket_32_40_T200", (32, 40, 200))):
        rel = torch.arange(T)[None, :] - torch.arange(T)[:, None]
        assert torch.equal(ref.relative_position_bucket(rel, nb, md)[0], fx[key])


@pytest.mark.slow
def test_large_dims_max_len_g10():
    """wav2vec2-Large dimensions (D 1024, 16 heads, FFN 4096, pre-norm, normalize_waveform), one utterance at
    lightning.py:313's max_len (250000 samples, T = 781 frames) plus a padded one."""
    fx = load_golden("g10_large.pt")
    out = _run_fixture(fx)
    assert out["student_hiddens"][0].shape == (2, 781, 1024)
    _check_step(fx, out, tol_loss=2e-5, tol_ck=5e-4)


def test_hubert_large_layer_norm_extractor_g11():
    """HuBERT-Large family (layer_norm extractor) at Large dimensions, all five pruning units."""
    fx = load_golden("g11_large_lnext.pt")
    out = _run_fixture(fx)
    _check_step(fx, out, tol_ck=2e-4)


def test_predlayer_mode_g12():
    """predlayer distill mode: independent Linear + GELU heads on the last student hidden state."""
    fx = load_golden("g12_predlayer.pt")
    assert fx["distill_mode"] == "predlayer"
    out = _run_fixture(fx)
    _check_step(fx, out)
    for n, ck in fx["proj_grad_ck"].items():
        # reference heads are nn.Sequential(Linear, GELU): "{i}.0.weight" is the oracle's "{i}.weight"
        e_sample, e_sq = ck_close(out["proj_grads"][n.replace(".0.", ".", 1)], ck)
        assert e_sample < 1e-4 and e_sq < 1e-4, (n, e_sample, e_sq)


@pytest.mark.slow
def test_large_24_layers_g13():
    """The full wav2vec2-Large depth of run_large.sh (24 pre-norm layers, distill layers 0.4,8,12,16,20,24)."""
    fx = load_golden("g13_large24.pt")
    out = _run_fixture(fx)
    assert len(out["student_hiddens"]) == 25
    _check_step(fx, out, tol_loss=2e-5, tol_ck=5e-4)
