"""Pruned (ragged) students on the GPU -- SURVEY §8f-1 (final_distill.py): per-layer head counts,
FFN widths and conv channel counts that are not multiples of 8, absent attention / FFN blocks.

The reference's own pruned model output is pinned by g4_prune.pt (hidden-state checksums of the
reference's prune() -> rebuilt model -> extract_features); the full final-distill step (teacher +
pruned student, no HardConcrete, fwd + bwd) is compared with the fp32 CPU oracle.
Tolerances: hidden sum-of-squares rel 2e-2 and sampled values 3e-2 of their scale (bf16
activations), loss 1e-3 abs (north star), parameter-gradient rel-L2 5e-2.
"""

import copy

import pytest
import torch

from dphubert_amd.cli import prune_config
from dphubert_amd.wav2vec2.model import wav2vec2_model
from helpers import ck_close, load_golden, proj_sd_from_recipe, rel_l2, seeded_sd, wave_batch
from oracle import hubert_ref as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pruned():
    fx = load_golden("g4_prune.pt")
    m = wav2vec2_model(**copy.deepcopy(fx["cfg"]))
    sd = seeded_sd(fx["cfg"], fx["seed"])
    sd.update(fx["log_alpha"])
    m.load_state_dict(sd)
    pcfg = prune_config(m, fx["cfg"])
    pm = wav2vec2_model(**copy.deepcopy(pcfg))
    pm.load_state_dict(m.state_dict(), strict=True)
    return fx, pcfg, pm


def test_pruned_shapes_are_ragged():
    fx, pcfg, _ = _pruned()
    widths = [c for c, _, _ in pcfg["extractor_conv_layer_config"]] + list(pcfg["encoder_ff_interm_features"])
    assert any(w % 8 for w in widths), widths


def test_pruned_forward_matches_reference():
    fx, pcfg, pm = _pruned()
    pm = pm.to(DEV).eval()
    with torch.no_grad():
        hs, _ = pm.extract_features(fx["wave"].to(DEV))
    torch.cuda.synchronize()
    assert len(hs) == len(fx["pruned_hidden_ck"])
    for h, ck in zip(hs, fx["pruned_hidden_ck"]):
        e_sample, e_sq = ck_close(h.float().cpu(), ck)
        assert e_sq < 2e-2 and e_sample < 3e-2, (e_sample, e_sq)


def test_final_distill_step_pruned_student_vs_oracle():
    from dphubert_amd.lightning import DistillLoss, DistillModule
    fx, pcfg, pm = _pruned()
    tcfg = {k: v for k, v in fx["cfg"].items()}
    for k in list(tcfg):
        if "_prune_" in k:
            tcfg[k] = False
    tsd = seeded_sd(tcfg, 1)
    teacher = wav2vec2_model(**copy.deepcopy(tcfg))
    teacher.load_state_dict(tsd)
    for p in teacher.parameters():
        p.requires_grad = False
    ssd = {k: v.detach().clone() for k, v in pm.state_dict().items()}
    psd = proj_sd_from_recipe(2, 768, 3)
    projs = []
    for g in range(2):
        lin = torch.nn.Linear(768, 768)
        with torch.no_grad():
            lin.weight.copy_(psd[f"{g}.weight"])
            lin.bias.copy_(psd[f"{g}.bias"])
        projs.append(lin)
    proj_index = [0, 1, 1]
    dm = DistillModule(teacher_model=teacher, student_model=pm, distill_mode="layer2layer", distill_layers=[0, 1, 2],
                       distill_linear_projs=torch.nn.ModuleList([projs[i] for i in proj_index]),
                       distill_loss=DistillLoss(0.0, 1.0, 1.0, "raw"), learning_rate=1e-4, weight_decay=0.0,
                       warmup_updates=5000, max_updates=25000, use_reg=False, reg_learning_rate=None,
                       target_sparsity=None, sparsity_warmup_updates=None).to(DEV)
    dm.train()
    wave, ln = wave_batch(2, 24000, seed=4, lengths=[24000, 19000])
    loss = dm._step((wave.to(DEV), ln.to(DEV)), 0, "train")
    loss.backward()
    torch.cuda.synchronize()
    want = ref.distill_step(tsd, tcfg, ssd, pcfg, psd, [0, 1, 2], proj_index, wave, ln, {}, None, 0)
    assert abs(loss.item() - want["loss"].item()) <= 1e-3, (loss.item(), want["loss"].item())
    got = dict(dm.student_model.named_parameters())
    checked = 0
    for n, g in want["grads"].items():
        if n not in got or got[n].grad is None or n.endswith("k_proj.bias") or g.norm() == 0:
            continue
        e = rel_l2(got[n].grad.float().cpu(), g)
        assert e < 5e-2, (n, e)
        checked += 1
    assert checked > 20


def test_bench_pruned_student_step_vs_oracle():
    """bench.py --student pruned's final_distill.py step (BASELINE config 4): HuBERT-Base teacher, the ~23.6 M-param
    student that synthetic.pruned_student prunes with the reference's prune() (ragged conv channels 101-122, 2-3 heads
    and 522-799 FFN units per layer), 12 layers at the bench's 10 s shape (T = 499), vs the fp32 CPU oracle."""
    from dphubert_amd.lightning import DistillLoss, DistillModule
    from dphubert_amd.synthetic import HUBERT_BASE_CONFIG, pruned_student
    tcfg = copy.deepcopy(HUBERT_BASE_CONFIG)
    tcfg.update(encoder_projection_dropout=0.0, encoder_attention_dropout=0.0, encoder_ff_interm_dropout=0.0,
                encoder_dropout=0.0, encoder_layer_drop=0.0)
    scfg, ssd = pruned_student(tcfg, seed=0)
    n = sum(v.numel() for v in ssd.values())
    assert abs(n - 23_585_946) < 0.01 * 23_585_946, n
    tsd = seeded_sd(tcfg, 0)
    teacher = wav2vec2_model(**copy.deepcopy(tcfg))
    teacher.load_state_dict(tsd)
    for p in teacher.parameters():
        p.requires_grad = False
    student = wav2vec2_model(**copy.deepcopy(scfg))
    student.load_state_dict(ssd, strict=True)
    psd = proj_sd_from_recipe(2, 768, 3)
    projs = []
    for g in range(2):
        lin = torch.nn.Linear(768, 768)
        with torch.no_grad():
            lin.weight.copy_(psd[f"{g}.weight"])
            lin.bias.copy_(psd[f"{g}.bias"])
        projs.append(lin)
    proj_index = [0, 1, 1, 1]
    layers = [0, 4, 8, 12]
    dm = DistillModule(teacher_model=teacher, student_model=student, distill_mode="layer2layer", distill_layers=layers,
                       distill_linear_projs=torch.nn.ModuleList([projs[i] for i in proj_index]),
                       distill_loss=DistillLoss(0.0, 1.0, 1.0, "raw"), learning_rate=1e-4, weight_decay=0.0,
                       warmup_updates=5000, max_updates=25000, use_reg=False, reg_learning_rate=None,
                       target_sparsity=None, sparsity_warmup_updates=None).to(DEV)
    dm.train()
    wave, ln = wave_batch(1, 160000, seed=6)
    loss = dm._step((wave.to(DEV), ln.to(DEV)), 0, "train")
    loss.backward()
    torch.cuda.synchronize()
    want = ref.distill_step(tsd, tcfg, ssd, scfg, psd, layers, proj_index, wave, ln, {}, None, 0)
    assert abs(loss.item() - want["loss"].item()) <= 1e-3, (loss.item(), want["loss"].item())
    got = dict(dm.student_model.named_parameters())
    checked = 0
    worst = (0.0, None)
    for n, g in want["grads"].items():
        if n not in got or got[n].grad is None or n.endswith("k_proj.bias") or g.norm() == 0:
            continue
        e = rel_l2(got[n].grad.float().cpu(), g)
        worst = max(worst, (e, n))
        assert e < 5e-2, (n, e)
        checked += 1
    print("pruned bench student: loss", loss.item(), "oracle", want["loss"].item(), "worst grad", worst)
    assert checked > 100
