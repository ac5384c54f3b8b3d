"""prune.py / save_final_ckpt.py path vs the reference's prune() run on the same
seeded weights and log_alpha (fixture g4_prune.pt): pruned architecture, pruned state_dict
checksums, and the checkpoint round trip of prune.py:13-73,100-105."""

import copy

import torch

from dphubert_amd.cli import load_pruned_model, prune_config, prune_from_ckpt, save_final_ckpt_main
from dphubert_amd.wav2vec2.model import wav2vec2_model
from helpers import ck_close, load_golden, seeded_sd


def _model(fx):
    m = wav2vec2_model(**copy.deepcopy(fx["cfg"]))
    sd = seeded_sd(fx["cfg"], fx["seed"])
    sd.update(fx["log_alpha"])
    m.load_state_dict(sd)
    return m


def test_prune_matches_reference():
    fx = load_golden("g4_prune.pt")
    m = _model(fx)
    pcfg = prune_config(m, fx["cfg"])
    assert [list(x) for x in pcfg["extractor_conv_layer_config"]] == fx["conv_config"]
    assert pcfg["encoder_use_attention"] == fx["use_attention"]
    assert pcfg["encoder_use_feed_forward"] == fx["use_feed_forward"]
    assert pcfg["encoder_num_heads"] == fx["num_heads"]
    assert pcfg["encoder_ff_interm_features"] == fx["ff_interm_features"]
    sd = m.state_dict()
    assert set(sd) == set(fx["state_dict_ck"])
    for k, ck in fx["state_dict_ck"].items():
        e_sample, e_sq = ck_close(sd[k], ck)
        assert e_sample < 1e-6 and e_sq < 1e-6, k
    # the pruned config rebuilds a model that takes the pruned weights strictly
    pm = wav2vec2_model(**copy.deepcopy(pcfg))
    pm.load_state_dict(sd, strict=True)


def test_prune_checkpoint_round_trip(tmp_path):
    fx = load_golden("g4_prune.pt")
    m = _model(fx)
    base_cfg = {k: v for k, v in fx["cfg"].items() if "_prune_" not in k}
    torch.save({"config": base_cfg, "state_dict": {}}, tmp_path / "orig.pth")
    lin = torch.nn.Linear(768, 768)
    distilled = {"student_model." + k: v for k, v in m.state_dict().items()}
    distilled.update({"distill_linear_projs.0.weight": lin.weight.detach(), "distill_linear_projs.0.bias":
                      lin.bias.detach(), "lambda1": torch.tensor(0.1)})
    torch.save({"state_dict": distilled, "global_step": 10}, tmp_path / "last.ckpt")
    out = prune_from_ckpt(tmp_path / "last.ckpt", tmp_path / "orig.pth")
    for k in ("extractor_conv_layer_config", "encoder_num_heads", "encoder_ff_interm_features",
              "encoder_use_attention", "encoder_use_feed_forward"):
        got = out["config"][k]
        want = fx["pruned_cfg"][k]
        assert [list(x) if isinstance(x, (list, tuple)) else x for x in got] == \
            [list(x) if isinstance(x, (list, tuple)) else x for x in want], k
    assert set(out["distill_linear_projs"]) == {"0.weight", "0.bias"}
    torch.save(out, tmp_path / "pruned_hubert_base.pth")
    pm = load_pruned_model(tmp_path / "pruned_hubert_base.pth")
    assert sum(p.numel() for p in pm.parameters()) < sum(p.numel() for p in m.parameters())
    # save_final_ckpt.py: config from the pruned file + weights of a final-distill checkpoint
    final = {"student_model." + k: v for k, v in out["state_dict"].items()}
    final.update({"distill_linear_projs." + k: v for k, v in out["distill_linear_projs"].items()})
    (tmp_path / "final").mkdir()
    torch.save({"state_dict": final}, tmp_path / "final" / "last.ckpt")
    save_final_ckpt_main(["--config_path", str(tmp_path / "pruned_hubert_base.pth"), "--ckpt_after_final_distill",
                          str(tmp_path / "final" / "last.ckpt")])
    pm2 = load_pruned_model(tmp_path / "final" / "pruned_hubert_base.pth")
    for (a, x), (b, y) in zip(pm.state_dict().items(), pm2.state_dict().items()):
        assert a == b and torch.equal(x, y)


def test_wavlm_prune_matches_reference():
    """WavLM prune (components.py:661-693: remaining_heads lists) vs the reference's prune() (fixture g9), and
    the oracle's forward of the pruned architecture vs the reference's pruned model on a padded batch."""
    from oracle import hubert_ref as ref
    fx = load_golden("g9_wavlm_prune.pt")
    m = _model(fx)
    pcfg = prune_config(m, fx["cfg"])
    assert pcfg["encoder_remaining_heads"] == fx["remaining_heads"]
    assert "encoder_num_heads" not in pcfg
    assert [list(x) for x in pcfg["extractor_conv_layer_config"]] == fx["conv_config"]
    assert pcfg["encoder_use_attention"] == fx["use_attention"]
    assert pcfg["encoder_ff_interm_features"] == fx["ff_interm_features"]
    sd = m.state_dict()
    assert set(sd) == set(fx["state_dict_ck"])
    for k, ck in fx["state_dict_ck"].items():
        e_sample, e_sq = ck_close(sd[k], ck)
        assert e_sample < 1e-6 and e_sq < 1e-6, k
    pm = wav2vec2_model(**copy.deepcopy(pcfg))
    pm.load_state_dict(sd, strict=True)
    psd = {k: v.detach() for k, v in sd.items()}
    with torch.no_grad():
        hs, _ = ref.extract_features(psd, pcfg, fx["wave"], fx["lengths"])
    for h, g in zip(hs, fx["pruned_hiddens"]):
        assert ((h - g).norm() / g.norm()).item() < 1e-5
