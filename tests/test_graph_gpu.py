"""Whole-step HIP-graph replay (trainer.Trainer(graphs=True)) against eager steps, and the
optimizer -> bf16 GEMM image hand-off.

Deterministic configuration (dropout 0, HardConcrete noise injected as device tensors) in the kernel library's
deterministic mode (include/dphubert_hip.h dph_set_deterministic: every cross-block float reduction in a fixed
order, no float atomics), so eager and replayed steps compute the same math in the same order: a replayed
trajectory must equal the eager one BITWISE -- every loss, every parameter after every optimizer step -- and two
eager runs must equal each other.  A short LR schedule (warmup 2, max 10 updates) makes every step use a different
learning rate, so the device-resident AdamW hyper-parameters are exercised.
"""

import copy
import os

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


def _module(seed=3, family="hubert", student_offset=True):
    """2-layer distill module.  ``student_offset``: the student's weights are the teacher's plus a seeded 10 %
    perturbation.  With student == teacher (run.sh:20's init) every distilled s - t starts at ~0, so the L1 term's
    gradient sign(s - t) is decided by rounding noise: after one AdamW update two EAGER runs already differ by
    1.7e-3 in their gradients (tools/graph_diag.py, profiles/r3_graph_diag_rccl_chaotic.txt) and no bound separates a
    stale op from that chaos.  Offset, the gradients are a smooth function of the weights."""
    from dphubert_amd.synthetic import seeded_tensor
    from dphubert_amd.trainer import build_distill_module
    dm = build_distill_module(_cfg(family), pruning_units="conv,head,interm", distill_layers="0.1,2", seed=seed,
                              learning_rate=2e-3, warmup_updates=2, max_updates=10, sparsity_warmup_updates=4)
    with torch.no_grad():
        dm.lambda1.fill_(0.3)
        dm.lambda2.fill_(0.2)
        if student_offset:
            for n, p in dm.student_model.named_parameters():
                if "log_alpha" not in n and p.numel() > 1:
                    p.add_(0.1 * p.abs().mean() * seeded_tensor("offset." + n, tuple(p.shape), seed + 1).sign())
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


@pytest.fixture(autouse=True)
def _deterministic():
    from dphubert_amd import _lib
    prev = _lib.deterministic()
    _lib.set_deterministic(True)
    yield
    _lib.set_deterministic(prev)


@pytest.mark.parametrize("family,accum", [("hubert", 1), ("wavlm", 1), ("large", 1), ("hubert", 3), ("large", 2)])
def test_graph_replay_matches_eager(family, accum):
    """Replayed steps equal eager steps bitwise (deterministic mode); accum > 1: first / middle / final micro-step
    graphs (run_large.sh:54 --accum_grad 3)."""
    from dphubert_amd.trainer import Trainer
    batch = _batch()
    # two eager runs (run-to-run determinism) and the graph run
    eager = [Trainer(_module(family=family), clip_norm=10.0, accum_grad=accum) for _ in range(2)]
    gr = Trainer(_module(family=family), clip_norm=10.0, graphs=True, graph_warmup=1, accum_grad=accum)
    le = [[] for _ in eager]
    lg = []
    for _ in range(5 * accum):
        for t, l in zip(eager, le):
            l.append(t.step(batch).item())
        lg.append(gr.step(batch).item())
    torch.cuda.synchronize()
    ea = eager[0]
    assert gr._graph is not None, "graph capture fell back to eager"
    assert len(gr._graphs) == min(accum, 3), sorted(gr._graphs)
    assert ea.module.global_step == gr.module.global_step == 1 + 5   # _module() starts at global_step 1
    assert len(set(round(x, 6) for x in lg)) > 1, "replayed steps did not train"
    _assert_bitwise(eager, gr, le, lg)
    # the graph replays follow the LR schedule: optimizer and scheduler state agree
    assert ea.optimizer._step == gr.optimizer._step
    for g1, g2 in zip(ea.optimizer.param_groups, gr.optimizer.param_groups):
        assert g1["lr"] == g2["lr"]


def bitwise_report(eager, gr, le, lg):
    """Deterministic mode: every eager run and the graph run must produce the same losses and the same parameters
    bit for bit (every parameter, k_proj.bias included).  Returns (ok, report lines naming each difference)."""
    ok, lines = True, []
    for i, l in enumerate(le[1:], 1):
        if l != le[0]:
            ok = False
            lines.append(f"eager run {i} losses {l} != eager run 0 {le[0]}")
    if lg != le[0]:
        ok = False
        lines.append(f"graph losses {lg} != eager {le[0]}")
    pg = dict(gr.module.named_parameters())
    for i, t in enumerate(eager):
        for n, p in t.module.named_parameters():
            if not torch.equal(p.detach(), pg[n].detach()):
                ok = False
                d = (p.detach().float() - pg[n].detach().float()).abs().max().item()
                lines.append(f"param {n}: eager run {i} vs graph max |diff| {d:.3g}")
    lines.append(f"{sum(1 for _ in pg)} parameters x {len(eager) + 1} runs compared bitwise; losses {lg}")
    return ok, lines


def _assert_bitwise(eager, gr, le, lg):
    ok, lines = bitwise_report(eager, gr, le, lg)
    assert ok, "\n".join(lines[:40])


def test_ffn_compaction_switch_under_graphs():
    """A gate whose expected zero fraction crosses Trainer.FFN_COMPACT_MIN_ZERO at a re-evaluation step under graph
    replay (a prune.py run toward 0.75 sparsity reaches it): the stale graphs are dropped, that optimizer step runs
    eagerly in the packed FFN layout, the next one recaptures -- and the trajectory tracks eager trainers making the
    same switch bitwise (deterministic mode)."""
    from dphubert_amd.trainer import Trainer
    batch = _batch()
    mk = lambda graphs: Trainer(_module(), clip_norm=10.0, graphs=graphs, graph_warmup=1)  # noqa: E731
    eager = [mk(False) for _ in range(2)]
    gr = mk(True)
    for t in eager + [gr]:
        t.FFN_COMPACT_EVERY = 3          # decisions at global steps 1, 4, 7 (_module() starts at 1)
    le = [[] for _ in eager]
    lg = []
    g = torch.Generator().manual_seed(5)
    for step in range(6):
        if step == 2:                    # before global step 3: half of layer 0's FFN units pushed to exact zeros
            n = gr.module.student_model.encoder.transformer.layers[0].feed_forward.hard_concrete_for_intermediate \
                .log_alpha.numel()
            idx = torch.randperm(n, generator=g)[: n // 2].to(DEV)
            for t in eager + [gr]:
                hc = t.module.student_model.encoder.transformer.layers[0].feed_forward.hard_concrete_for_intermediate
                with torch.no_grad():
                    hc.log_alpha[idx] = -10.0
        for t, l in zip(eager, le):
            l.append(t.step(batch).item())
        lg.append(gr.step(batch).item())
        if step == 3:                    # global step 4: the switch -- graphs dropped, this step eager
            assert not gr._graphs and gr._eager_until == 5
    torch.cuda.synchronize()
    hc = gr.module.student_model.encoder.transformer.layers[0].feed_forward.hard_concrete_for_intermediate
    assert getattr(hc, "dph_compact", False), "the gate did not switch to the packed FFN"
    assert gr._graph is not None, "no graph recaptured after the switch"
    _assert_bitwise(eager, gr, le, lg)


def test_profiled_graph_survives_grouped_fallback(monkeypatch):
    """Round-3 host segfault in the profiled step replay (gpurun_out/r3_s25): a grouped weight-gradient launch that
    returned DPH_EUNSUPPORTED after its start event was recorded into the graph dropped that event, and the replay
    recorded a destroyed hipEvent.  Every grouped launch is forced to fall back here; the profiler owns its events,
    so the replays after a garbage collection run and time every GEMM."""
    import gc
    from dphubert_amd import _lib
    from dphubert_amd import kernels as K
    from dphubert_amd.kernels import LaunchProfiler
    from dphubert_amd.trainer import Trainer
    batch = _batch()
    tr = Trainer(_module(), clip_norm=10.0, graphs=True, graph_warmup=1)
    for _ in range(2):
        tr.step(batch)
    monkeypatch.setattr(_lib.lib(), "dph_gemm_grouped", lambda *a: K.EUNSUPPORTED)
    prof = LaunchProfiler()
    tr.prepare_profiled_step(prof)
    assert len(prof.events) > 2 * len(prof.records), "no grouped launch fell back"
    gc.collect()
    for _ in range(2):
        loss = tr.step(batch, profiled=True)
    torch.cuda.synchronize()
    assert torch.isfinite(loss).item()
    summ = prof.summary()
    assert summ and all(v["ms"] > 0 for v in summ.values()), summ


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


@pytest.mark.parametrize("comm,accum", [("fp32", 1), ("bf16", 2)])
def test_graph_replay_with_rccl_allreduce(comm, accum):
    """The whole-step graph with the RCCL gradient all-reduce captured inside it (world size 1 over the
    "nccl" = RCCL backend, the reducer forced on so every bucket really goes through RCCL): replayed
    optimizer steps match eager steps; bf16 payload and accumulation (first / final micro-step graphs)
    too.  Runs tools/graph_rccl_probe.py in a child process (its own process group)."""
    import socket
    import subprocess
    import sys
    from pathlib import Path
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, str(root / "tools" / "graph_rccl_probe.py"), "--comm", comm, "--accum",
                        str(accum), "--port", str(port)], capture_output=True, text=True, timeout=240, env=env,
                       cwd=str(root))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "RCCL_GRAPH_OK" in out, out[-3000:]


def test_grouped_wgrads_match_per_layer(monkeypatch):
    """Encoder-layer weight gradients deferred and launched as grouped GEMMs (ops.grouped_wgrads: group 2 over the
    2-layer model, so every layer kind lands in one dph_gemm_grouped launch) against one launch per layer: the
    same gradient buckets up to fp32 summation order (the grouped plan needs fewer split-K slices)."""
    from dphubert_amd import kernels as K
    from dphubert_amd.trainer import Trainer
    batch = _batch()
    calls = []
    orig = K.linear_wgrad_grouped

    def spy(items, **kw):
        calls.append(len(items))
        return orig(items, **kw)

    monkeypatch.setattr(K, "linear_wgrad_grouped", spy)
    res = []
    for g in (1, 2):
        monkeypatch.setenv("DPH_WGRAD_GROUP", str(g))
        tr = Trainer(_module(), clip_norm=10.0)
        tr.step(batch)
        torch.cuda.synchronize()
        res.append(torch.cat([f.detach().float().cpu() for f in tr.reducer.flat]))
        assert not any(getattr(p, "_dph_hold", False) for p in tr.reducer.params)
    assert calls == [2, 2, 2, 2], calls     # FFN w2, FFN w1, out-proj, qkv: both layers each
    assert rel_l2(res[1], res[0]) < 1e-4


@pytest.mark.parametrize("family", ["hubert", "wavlm", "large"])
def test_deterministic_mode_matches_atomic_reductions(family):
    """The fixed-order reductions of deterministic mode (LayerNorm-affine / bias column sums, mask gradients, conv0
    sums, head-mask sums, the WavLM diagonal and gate sums) against the float-atomic ones: one step's gradients agree
    to fp32 summation-order noise (whole gradient vector rel-L2 < 1e-5), and deterministic mode repeats bitwise."""
    from dphubert_amd import _lib
    from dphubert_amd.ddp import GradReducer
    batch = _batch()
    grads = []
    for det in (True, False, True):
        _lib.set_deterministic(det)
        dm = _module(family=family)
        red = GradReducer([p for p in dm.parameters() if p.requires_grad])
        red.prepare()
        loss = dm._step(batch, 0, "train")
        loss.backward()
        red.finish()
        torch.cuda.synchronize()
        grads.append(torch.cat([f.detach().float().cpu() for f in red.flat]))
        red.remove()
    assert torch.equal(grads[0], grads[2]), "deterministic mode did not repeat bitwise"
    assert rel_l2(grads[1], grads[0]) < 1e-5, rel_l2(grads[1], grads[0])


@pytest.mark.parametrize("group", [1, 2])
def test_ffn_mask_grad_colprod_matches_epilogue(monkeypatch, group):
    """the FFN intermediate-mask gradient from the FFN2 weight gradient (dph_colprod: sum_o W2[o][n]
    dW2[o][n] / mask_n, the default) against the f-reading DGK epilogue (DPH_FFN_COLPROD=0), ungrouped and grouped
    weight gradients, over two accumulated micro-batches (the second one takes the epilogue either way: its bucket
    is no longer fresh), with intermediate masks exactly 0, near 0 and near 1."""
    from dphubert_amd import ops
    from dphubert_amd.ddp import GradReducer
    batch = _batch()
    res = []
    for colprod in (True, False):
        monkeypatch.setattr(ops, "_FFN_COLPROD", colprod)
        dm = _module()
        g = torch.Generator().manual_seed(3)
        for name, mod in dm.student_model.named_modules():
            if name.endswith("hard_concrete_for_intermediate"):
                n = mod.log_alpha.numel()
                u = torch.rand(n, generator=g) * 0.98 + 0.01
                u[: n // 4] = 1e-4            # sampled below 0: clamped to exactly 0 (hardconcrete.py:99)
                u[n // 4: n // 2] = 0.9999     # near 1
                mod.set_noise(u.to(DEV))
        red = GradReducer([p for p in dm.parameters() if p.requires_grad])
        grads = []
        for micro in range(2):
            red.prepare(zero=micro == 0, sync=micro == 1)
            with ops.grouped_wgrads(group):
                (dm._step(batch, 0, "train") / 2).backward()
            torch.cuda.synchronize()
            grads.append({n: p.grad.detach().clone().cpu() for n, p in dm.student_model.named_parameters()
                          if n.endswith("hard_concrete_for_intermediate.log_alpha")})
        red.finish()
        red.remove()
        res.append(grads)
    for micro in range(2):
        for n, a in res[0][micro].items():
            b = res[1][micro][n]
            assert rel_l2(a, b) < 1e-4, (micro, n, rel_l2(a, b))


@pytest.mark.parametrize("accum", [1, 2])
def test_deferred_reductions_match_immediate(monkeypatch, accum):
    """ops.deferred_reductions (the sink-bound bias / LayerNorm-affine column reductions queued by the library and
    launched as one grid at the encoder-end flush) against immediate launches: the same gradient buckets BITWISE
    (each queued problem is summed in the fixed order of its own launch), reductions really queued, and no
    parameter left held back from the reducer."""
    from dphubert_amd import _lib, ops
    from dphubert_amd.trainer import Trainer
    batch = _batch()
    queued = []
    orig = ops.deferred_reductions.close

    def spy(self):
        if self.open:
            queued.append(_lib.lib().dph_deferred_reductions())
        return orig(self)

    monkeypatch.setattr(ops.deferred_reductions, "close", spy)
    res = []
    for on in ("0", "1"):
        monkeypatch.setenv("DPH_DEFER_RED", on)
        tr = Trainer(_module(), clip_norm=10.0, accum_grad=accum)
        for _ in range(accum):
            tr.step(batch)
        torch.cuda.synchronize()
        res.append(torch.cat([f.detach().float().cpu() for f in tr.reducer.flat]))
        assert not any(getattr(p, "_dph_hold", False) for p in tr.reducer.params)
        assert _lib.lib().dph_deferred_reductions() == 0
    assert queued and max(queued) >= 8, queued
    assert torch.equal(res[0], res[1])


def test_deferred_block_error_discards_queue(monkeypatch):
    """A deferred_reductions block left by an exception (e.g. a HIP-graph capture that raised: trainer.py falls back
    to eager steps) drops its queued reductions unlaunched: their slabs are no longer kept and their sinks belong to
    an abandoned step.  The next step's gradient buckets must equal an immediate-mode step BITWISE (a stale queue
    flushed into them would add the abandoned step's partial sums)."""
    from dphubert_amd import _lib, ops
    from dphubert_amd import kernels as K
    from dphubert_amd.trainer import Trainer
    batch = _batch()
    seen = []

    def boom(grad):
        seen.append(int(_lib.lib().dph_deferred_reductions()))
        raise RuntimeError("injected failure inside the deferred block")

    monkeypatch.setenv("DPH_DEFER_RED", "1")
    tr = Trainer(_module(), clip_norm=10.0)
    monkeypatch.setattr(ops, "_flush_wgrads_hook", boom)
    with pytest.raises(RuntimeError, match="injected failure"):
        tr.step(batch)
    monkeypatch.undo()
    assert seen and seen[0] > 0, seen                       # reductions were queued when the block failed
    assert _lib.lib().dph_deferred_reductions() == 0        # ... and dropped, not left for a later flush
    assert not K.ARMED[0] and K.KEEP_WS[0] is None
    tr._micro = 0
    tr.step(batch)                                          # same weights: the failed step updated nothing
    torch.cuda.synchronize()
    got = torch.cat([f.detach().float().cpu() for f in tr.reducer.flat])
    monkeypatch.setenv("DPH_DEFER_RED", "0")
    ref = Trainer(_module(), clip_norm=10.0)
    ref.step(batch)
    torch.cuda.synchronize()
    want = torch.cat([f.detach().float().cpu() for f in ref.reducer.flat])
    assert torch.equal(got, want)
