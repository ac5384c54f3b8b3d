"""Whole-step HIP-graph replay (trainer.Trainer(graphs=True)) against eager steps, and the
optimizer -> bf16 GEMM image hand-off.

Deterministic configuration (dropout 0, HardConcrete noise injected as device tensors) so that eager
and replayed steps compute the same math; the remaining differences are fp32 atomics in weight/bias
gradient reductions (~1e-6 relative).  A short LR schedule (warmup 2, max 10 updates) makes every
step use a different learning rate, so the device-resident AdamW hyper-parameters are exercised.
"""

import copy

import pytest
import torch

from helpers import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _cfg(family="hubert"):
    from dphubert_amd.synthetic import HUBERT_BASE_CONFIG, WAVLM_BASE_CONFIG
    if family == "large":
        # HuBERT-Large family at Large width (convert_hubert_large_from_fairseq.py:19-40): layer_norm extractor,
        # pre-norm layers, normalize_waveform (its crop length is replayed from the eager step)
        cfg = copy.deepcopy(HUBERT_BASE_CONFIG)
        cfg.update(extractor_mode="layer_norm", encoder_embed_dim=1024, encoder_num_heads=[16] * 2,
                   encoder_layer_norm_first=True, normalize_waveform=True)
        cfg.update(encoder_num_layers=2, encoder_use_attention=[True] * 2, encoder_use_feed_forward=[True] * 2,
                   encoder_ff_interm_features=[4096] * 2, encoder_projection_dropout=0.0,
                   encoder_attention_dropout=0.0, encoder_ff_interm_dropout=0.0, encoder_dropout=0.0,
                   encoder_layer_drop=0.0)
        return cfg
    if family == "wavlm":
        # WavLM: the relative-position table, gate and their gradients run inside the captured graph too
        cfg = copy.deepcopy(WAVLM_BASE_CONFIG)
        cfg.update(encoder_total_num_heads=[12] * 2, encoder_remaining_heads=[list(range(12))] * 2)
    else:
        cfg = copy.deepcopy(HUBERT_BASE_CONFIG)
        cfg.update(encoder_num_heads=[12] * 2)
    cfg.update(encoder_num_layers=2, encoder_use_attention=[True] * 2, encoder_use_feed_forward=[True] * 2,
               encoder_ff_interm_features=[3072] * 2, encoder_projection_dropout=0.0,
               encoder_attention_dropout=0.0, encoder_ff_interm_dropout=0.0, encoder_dropout=0.0,
               encoder_layer_drop=0.0)
    return cfg


def _module(seed=3, family="hubert"):
    from dphubert_amd.trainer import build_distill_module
    dm = build_distill_module(_cfg(family), pruning_units="conv,head,interm", distill_layers="0.1,2", seed=seed,
                              learning_rate=2e-3, warmup_updates=2, max_updates=10, sparsity_warmup_updates=4)
    with torch.no_grad():
        dm.lambda1.fill_(0.3)
        dm.lambda2.fill_(0.2)
    dm.global_step = 1
    g = torch.Generator().manual_seed(11)
    dm = dm.to(DEV)
    for name, mod in dm.student_model.named_modules():
        if hasattr(mod, "set_noise"):
            mod.set_noise((torch.rand(mod.log_alpha.shape, generator=g) * 0.98 + 0.01).to(DEV))
    return dm


def _batch():
    from dphubert_amd.synthetic import synthetic_batch
    w, l = synthetic_batch(2, 16000)
    l[1] = 12000
    w[1, 12000:] = 0
    return w.to(DEV), l.to(DEV)


def test_optimizer_updates_reach_gemm_images():
    """After an optimizer step the student's forward must use the UPDATED weights (the fused AdamW
    writes the fp32 masters behind autograd's back and bumps their versions)."""
    from dphubert_amd.trainer import Trainer
    dm = _module()
    tr = Trainer(dm, clip_norm=10.0)
    batch = _batch()
    tr.step(batch)
    tr.step(batch)
    torch.cuda.synchronize()
    fresh = copy.deepcopy(dm.student_model)
    fresh.load_state_dict({k: v.detach().clone() for k, v in dm.student_model.state_dict().items()})
    for m in (dm.student_model, fresh):
        m.eval()
    with torch.no_grad():
        h1, _ = dm.student_model.extract_features(*batch)
        h2, _ = fresh.extract_features(*batch)
    torch.cuda.synchronize()
    for a, b in zip(h1, h2):
        assert torch.equal(a, b)


@pytest.mark.parametrize("family,accum", [("hubert", 1), ("wavlm", 1), ("large", 1), ("hubert", 3), ("large", 2)])
def test_graph_replay_matches_eager(family, accum):
    """Replayed steps track eager steps as closely as two eager runs track each other (the only
    run-to-run difference is the fp32 atomic order of gradient reductions, which AdamW's
    normalisation amplifies on tiny gradients).  accum > 1: first / middle / final micro-step graphs
    (run_large.sh:54 --accum_grad 3)."""
    from dphubert_amd.trainer import Trainer
    batch = _batch()
    ea = Trainer(_module(family=family), clip_norm=10.0, accum_grad=accum)
    eb = Trainer(_module(family=family), clip_norm=10.0, accum_grad=accum)
    gr = Trainer(_module(family=family), clip_norm=10.0, graphs=True, graph_warmup=1, accum_grad=accum)
    le, lb, lg = [], [], []
    for _ in range(5 * accum):
        le.append(ea.step(batch).item())
        lb.append(eb.step(batch).item())
        lg.append(gr.step(batch).item())
    torch.cuda.synchronize()
    assert gr._graph is not None, "graph capture fell back to eager"
    assert len(gr._graphs) == min(accum, 3), sorted(gr._graphs)
    assert ea.module.global_step == gr.module.global_step == 1 + 5   # _module() starts at global_step 1
    # losses: as close as two eager runs are (fp32 atomic order in weight-gradient reductions,
    # amplified by Adam over the steps) plus 1e-4
    for a, b, c in zip(le, lg, lb):
        assert abs(a - b) <= 1e-4 * max(1.0, abs(a)) + 4 * abs(a - c), (le, lg, lb)
    assert len(set(round(x, 6) for x in lg)) > 1, "replayed steps did not train"
    pa = dict(ea.module.named_parameters())
    pb = dict(eb.module.named_parameters())
    names = [n for n, p in gr.module.named_parameters() if p.requires_grad and not n.endswith("k_proj.bias")]
    # k_proj.bias has an exactly-zero gradient (softmax shift invariance): Adam turns the fp32
    # atomic-order noise of that zero into +-lr steps, so it is not comparable run to run.
    # Per parameter: within 4x the eager-vs-eager drift of the same parameter or 5e-3; 1-D biases
    # 1e-2 (their gradients are column sums with heavy cancellation, so Adam's normalised step
    # turns atomic-order noise into drift of 2e-3..7e-3 between two EAGER runs after 5 steps, and
    # one eager pair is a noisy estimate of that spread); all parameters together: within 4x the
    # eager-vs-eager drift of the whole parameter vector.
    pg = dict(gr.module.named_parameters())
    for n in names:
        e = rel_l2(pg[n].detach().cpu(), pa[n].detach().cpu())
        base = rel_l2(pb[n].detach().cpu(), pa[n].detach().cpu())
        floor = 1e-2 if pg[n].dim() == 1 else 5e-3
        assert e < max(floor, 4 * base), (n, e, base)
    cat = lambda d: torch.cat([d[n].detach().float().flatten().cpu() for n in names])  # noqa: E731
    e_all, base_all = rel_l2(cat(pg), cat(pa)), rel_l2(cat(pb), cat(pa))
    assert e_all < max(1e-5, 4 * base_all), (e_all, base_all)
    # the graph replays follow the LR schedule: optimizer and scheduler state agree
    assert ea.optimizer._step == gr.optimizer._step
    for g1, g2 in zip(ea.optimizer.param_groups, gr.optimizer.param_groups):
        assert g1["lr"] == g2["lr"]


def test_graph_profiled_step_events():
    from dphubert_amd.kernels import LaunchProfiler
    from dphubert_amd.trainer import Trainer
    batch = _batch()
    tr = Trainer(_module(), clip_norm=10.0, graphs=True, graph_warmup=1)
    for _ in range(2):
        tr.step(batch)
    prof = LaunchProfiler()
    tr.prepare_profiled_step(prof)
    loss = tr.step(batch, profiled=True)
    torch.cuda.synchronize()
    assert torch.isfinite(loss).item()
    summ = prof.summary()
    assert summ and all(v["ms"] > 0 and v["launches"] > 0 for v in summ.values()), summ
