"""The headline shape in graph mode (BASELINE config 2): HuBERT-Base teacher + student, 12 layers, B = 16 x 10 s,
distill layers ``0.4,8,12``, HardConcrete conv,head,interm with injected noise, dropout 0.

A graph trainer (2 eager warm-up steps, then the captured main step graph, then the profiled -- event-node --
step graph that bench.py replays for its roofline) runs in lockstep with an eager trainer from the same seeded
state, in the kernel library's deterministic mode (dph_set_deterministic).  Every step's loss terms
(lightning.py:245-296: loss, distill, l1, cos, reg) and the expected sparsity (model.py:109-113) must EQUAL the
eager step's, and after the last step every parameter must equal the eager trainer's bit for bit: a replay that
reads stale memory or whose accumulators are overwritten departs at once.
"""

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _module():
    from dphubert_amd.synthetic import HUBERT_BASE_CONFIG
    from dphubert_amd.trainer import build_distill_module
    cfg = copy.deepcopy(HUBERT_BASE_CONFIG)
    cfg.update(encoder_projection_dropout=0.0, encoder_attention_dropout=0.0, encoder_ff_interm_dropout=0.0,
               encoder_dropout=0.0, encoder_layer_drop=0.0)
    dm = build_distill_module(cfg, pruning_units="conv,head,interm", distill_layers="0.4,8,12", use_reg=True)
    with torch.no_grad():
        dm.lambda1.fill_(0.3)
        dm.lambda2.fill_(0.2)
    dm.global_step = 5000                   # target sparsity 0.75 (bench setting)
    dm = dm.to(DEV)
    g = torch.Generator().manual_seed(7)
    for _, mod in dm.student_model.named_modules():
        if hasattr(mod, "set_noise"):
            mod.set_noise((torch.rand(mod.log_alpha.shape, generator=g) * 0.98 + 0.01).to(DEV))
    return dm


TERMS = ("train_loss", "train_loss_distill", "train_loss_l1", "train_loss_cos", "train_loss_reg")


def _terms(dm):
    out = {k: float(dm.logged[k]) for k in TERMS}
    out["sparsity_expected"] = float(dm.logged["sparsity_expected"])
    return out


def test_headline_shape_graph_matches_eager():
    from dphubert_amd import _lib
    from dphubert_amd.kernels import LaunchProfiler
    from dphubert_amd.synthetic import synthetic_batch
    from dphubert_amd.trainer import Trainer
    _lib.set_deterministic(True)
    w, l = synthetic_batch(16, 160000)
    batch = (w.to(DEV), l.to(DEV))
    te = Trainer(_module(), clip_norm=10.0)
    tg = Trainer(_module(), clip_norm=10.0, graphs=True, graph_warmup=2)
    # graph trainer: eager, eager, capture+main replay, main, profiled, main, profiled
    plan = ["eager", "eager", "main", "main", "prof", "main", "prof"]
    seen = []
    for i, kind in enumerate(plan):
        if kind == "prof" and tg._prof_graph is None:
            tg.prepare_profiled_step(LaunchProfiler())
        le = te.step(batch)
        lg = tg.step(batch, profiled=(kind == "prof"))
        torch.cuda.synchronize()
        if kind != "eager":
            assert tg._graph is not None, "graph capture fell back to eager"
        e, g = _terms(te.module), _terms(tg.module)
        assert abs(le.item() - e["train_loss"]) < 1e-7 and abs(lg.item() - g["train_loss"]) < 1e-7
        seen.append((kind, e, g))
        for k in TERMS:
            assert g[k] == g[k] and abs(g[k]) < 1e3, (i, kind, k, g)            # finite, sane magnitude
            assert g[k] == e[k], (i, kind, k, e[k], g[k], seen)
        assert g["train_loss_l1"] > 0.0, (i, kind, g)
        assert g["sparsity_expected"] == e["sparsity_expected"], (i, kind, e, g)
    assert te.module.global_step == tg.module.global_step == 5000 + len(plan)
    pe = dict(te.module.named_parameters())
    bad = [n for n, p in tg.module.named_parameters() if not torch.equal(p.detach(), pe[n].detach())]
    assert not bad, bad[:20]
