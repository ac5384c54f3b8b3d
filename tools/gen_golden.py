"""Generate golden parity fixtures by importing the REFERENCE (build container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py

The reference (/root/reference, read-only) is imported in-process with two
light stubs injected into sys.modules (pytorch_lightning and torchaudio are not
installed).  Nothing from the reference is copied: the outputs
written to tests/golden/*.pt are pure data (inputs, expected outputs,
checksums) loadable with ``torch.load(..., weights_only=True)``.

Weights come from dphubert_amd.synthetic.seeded_tensor, so the tests rebuild
the exact same fp32 parameters without shipping a checkpoint.  HardConcrete
noise ``u`` is recorded by wrapping ``Tensor.uniform_`` while each
HardConcrete module runs, so the oracle can replay it.
"""

import copy
import os
import sys
import types
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[1]
REF = Path("/root/reference")
OUT = REPO / "tests" / "golden"
sys.path.insert(0, str(REPO))
sys.dont_write_bytecode = True

from dphubert_amd.synthetic import HUBERT_BASE_CONFIG, seeded_tensor  # noqa: E402


def _install_stubs():
    pl = types.ModuleType("pytorch_lightning")

    class LightningModule(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.global_step = 0
            self.logged = {}

        def log_dict(self, d, **kw):
            self.logged.update({k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in d.items()})

    pl.LightningModule = LightningModule
    cb = types.ModuleType("pytorch_lightning.callbacks")
    cb.ModelCheckpoint = object
    cb.LearningRateMonitor = object
    pl.callbacks = cb
    sys.modules["pytorch_lightning"] = pl
    sys.modules["pytorch_lightning.callbacks"] = cb
    ta = types.ModuleType("torchaudio")
    sys.modules["torchaudio"] = ta


_install_stubs()
sys.path.insert(0, str(REF))
from wav2vec2.model import wav2vec2_model  # noqa: E402  (reference)
from wav2vec2.hardconcrete import HardConcrete  # noqa: E402  (reference)
import lightning as ref_lightning  # noqa: E402  (reference)


def checksum(t: torch.Tensor) -> dict:
    t = t.detach().double().flatten()
    n = t.numel()
    idx = torch.linspace(0, n - 1, min(64, n)).long()
    return {"n": n, "sum": t.sum().item(), "abs": t.abs().sum().item(), "sq": (t * t).sum().item(),
            "head": t[:16].float().clone(), "sample_idx": idx, "sample": t[idx].float().clone()}


def seeded_model(cfg, seed):
    m = wav2vec2_model(**copy.deepcopy(cfg))
    sd = {k: seeded_tensor(k, v.shape, seed) for k, v in m.state_dict().items()}
    m.load_state_dict(sd, strict=True)
    return m, sd


class URecorder:
    """Record HardConcrete noise u per module (in call order)."""

    def __init__(self, model):
        self.cur = None
        self.u = {}
        self.hooks = []
        for name, mod in model.named_modules():
            if isinstance(mod, HardConcrete):
                self.hooks.append(mod.register_forward_pre_hook(self._pre(name)))

    def _pre(self, name):
        def f(mod, inp):
            self.cur = name
        return f

    def __enter__(self):
        self._orig = torch.Tensor.uniform_
        rec = self

        def uniform_(t, *a, **k):
            r = rec._orig(t, *a, **k)
            if rec.cur is not None:
                rec.u[rec.cur] = t.detach().clone()
                rec.cur = None
            return r

        torch.Tensor.uniform_ = uniform_
        return self

    def __exit__(self, *exc):
        torch.Tensor.uniform_ = self._orig
        for h in self.hooks:
            h.remove()


def no_dropout(cfg):
    c = copy.deepcopy(cfg)
    c.update(encoder_projection_dropout=0.0, encoder_attention_dropout=0.0, encoder_ff_interm_dropout=0.0,
             encoder_dropout=0.0, encoder_layer_drop=0.0)
    return c


def small_cfg(n_layers, **kw):
    c = no_dropout(HUBERT_BASE_CONFIG)
    c.update(encoder_num_layers=n_layers, encoder_use_attention=[True] * n_layers,
             encoder_use_feed_forward=[True] * n_layers, encoder_num_heads=[12] * n_layers,
             encoder_ff_interm_features=[3072] * n_layers)
    c.update(kw)
    return c


def units_flags(units):
    return dict(extractor_prune_conv_channels="conv" in units, encoder_prune_attention_heads="head" in units,
                encoder_prune_attention_layer="attlayer" in units,
                encoder_prune_feed_forward_intermediate="interm" in units,
                encoder_prune_feed_forward_layer="ffnlayer" in units)


def wave_batch(B, S, seed=2022, lengths=None):
    g = torch.Generator()
    g.manual_seed(seed)
    w = 0.1 * torch.randn(B, S, generator=g)
    if lengths is None:
        lengths = [S] * B
    ln = torch.tensor(lengths, dtype=torch.int64)
    for b, l in enumerate(lengths):
        w[b, l:] = 0.0
    return w, ln


class Bf16Emulation:
    """Run the reference's nn.Linear / nn.Conv1d layers the way a bf16-operand GEMM path does: input, weight and
    output rounded to bf16 in the forward (straight-through), the gradients leaving the layer (input gradient) and
    arriving at it (output gradient) rounded to bf16 in the backward; and the attention probabilities the way a
    flash kernel with bf16 MFMA operands does: P rounded to bf16 before P @ V, the score gradient dS rounded to bf16
    before dS @ K / dS^T @ Q.  Used only to MEASURE how sensitive each fixture quantity is to bf16 arithmetic (the
    fixture's expected values always come from the exact fp32 run)."""

    @staticmethod
    def _r(t, grad_round=True):
        tr = t.detach().to(torch.bfloat16).float()
        out = t + (tr - t.detach())
        if grad_round and out.requires_grad:
            out.register_hook(lambda g: g.to(torch.bfloat16).float())
        return out

    def __enter__(self):
        self.orig = (torch.nn.Linear.forward, torch.nn.Conv1d.forward, torch.nn.functional.softmax,
                     torch.nn.functional.layer_norm)
        r = self._r
        softmax = self.orig[2]
        layer_norm = self.orig[3]

        def ln(x, *a, **k):       # bf16 activations in HBM: the LayerNorm reads and writes bf16 rows
            return r(layer_norm(r(x), *a, **k))

        def sm(x, *a, **k):
            if x.requires_grad:
                x.register_hook(lambda g: g.to(torch.bfloat16).float())     # dS
            return r(softmax(x, *a, **k), False)                                # P (bf16 MFMA operand)

        def lin(mod, x):
            return r(torch.nn.functional.linear(r(x), r(mod.weight, False), mod.bias))

        def conv(mod, x):
            return r(mod._conv_forward(r(x), r(mod.weight, False), mod.bias))

        torch.nn.Linear.forward = lin
        torch.nn.Conv1d.forward = conv
        torch.nn.functional.softmax = sm
        torch.nn.functional.layer_norm = ln
        return self

    def __exit__(self, *exc):
        (torch.nn.Linear.forward, torch.nn.Conv1d.forward, torch.nn.functional.softmax,
         torch.nn.functional.layer_norm) = self.orig


def _ck_err(a, b):
    """(rel-L2 of the sampled entries, max sampled error / max sampled magnitude, relative sum of squares) of
    checksum a against checksum b."""
    sa, sb = a["sample"].double(), b["sample"].double()
    rl2 = ((sa - sb).norm() / sb.norm().clamp_min(1e-30)).item()
    mx = ((sa - sb).abs().max() / (sb.abs().max() + 1e-6)).item()
    sq = abs(a["sq"] - b["sq"]) / max(b["sq"], 1e-30)
    return (rl2, mx, sq)


def bf16_sensitivity(exact, emulated):
    """How far each fixture quantity moves when the reference itself runs with bf16-rounded GEMM outputs and
    activation gradients: the conditioning the GPU parity tolerances are scaled by (tests/test_parity_gpu.py)."""
    rl2 = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()  # noqa: E731
    return {
        "loss": abs(emulated["loss"].item() - exact["loss"].item()),
        "grad": {n: _ck_err(emulated["grad_ck"][n], ck) for n, ck in exact["grad_ck"].items()},
        "proj_grad": {n: _ck_err(emulated["proj_grad_ck"][n], ck) for n, ck in exact["proj_grad_ck"].items()},
        "log_alpha": {n: rl2(emulated["log_alpha_grads"][n], g) for n, g in exact["log_alpha_grads"].items()},
        "hidden": [_ck_err(a, b) for a, b in zip(emulated["student_hidden_ck"], exact["student_hidden_ck"])],
    }


def run_step(tcfg, scfg, distill_layers_str, B, S, units, lambdas, global_step, seed=0, lengths=None,
             full=False, cos_type="raw", l2=0.0, distill_mode="layer2layer", sens=True, whole=None):
    """Run the reference DistillModule._step + backward; return a fixture dict (plus, with ``sens``, the bf16
    sensitivity of every checked quantity from a second run under Bf16Emulation with the same noise).

    ``whole``: a predicate on student parameter names whose gradients are stored WHOLE (bf16 values plus their
    exact fp32 norm, and their bf16-emulation sensitivity as a whole-tensor rel-L2)."""
    if sens:
        kw = dict(seed=seed, lengths=lengths, full=full, cos_type=cos_type, l2=l2, distill_mode=distill_mode,
                  sens=False, whole=whole)
        fx = run_step(tcfg, scfg, distill_layers_str, B, S, units, lambdas, global_step, **kw)
        with Bf16Emulation():
            em = run_step(tcfg, scfg, distill_layers_str, B, S, units, lambdas, global_step, **kw)
        fx["sens"] = bf16_sensitivity(fx, em)
        if whole is not None:
            rl2 = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()  # noqa
            fx["sens"]["whole"] = {n: rl2(em["whole_f32"][n], g) for n, g in fx["whole_f32"].items()}
            fx["whole_grads"] = {n: g.to(torch.bfloat16) for n, g in fx["whole_f32"].items()}
            fx["whole_norms"] = {n: g.double().norm().item() for n, g in fx["whole_f32"].items()}
            del fx["whole_f32"]
        return fx
    scfg = dict(scfg, **units_flags(units))
    teacher, tsd = seeded_model(tcfg, seed)
    student, ssd = seeded_model(scfg, seed)   # student init = teacher weights (run.sh:20) + seeded log_alpha
    for p in teacher.parameters():
        p.requires_grad = False
    groups = [[int(x) for x in g.split(",")] for g in distill_layers_str.split(".")]
    layers, projs, proj_index = [], torch.nn.ModuleList(), []
    D = scfg["encoder_embed_dim"]
    proj_sd = {}
    if distill_mode == "layer2layer":
        for gi, g in enumerate(groups):
            lin = torch.nn.Linear(D, tcfg["encoder_embed_dim"])
            # identity init (distill.py:24-26) perturbed by a seeded delta so grads are non-trivial
            with torch.no_grad():
                lin.weight.copy_(torch.eye(D) + seeded_tensor(f"proj{gi}.weight", (D, D), seed) * 0.05)
                lin.bias.copy_(seeded_tensor(f"proj{gi}.bias", (D,), seed))
            proj_sd[f"{gi}.weight"] = lin.weight.detach().clone()
            proj_sd[f"{gi}.bias"] = lin.bias.detach().clone()
            for l in g:
                layers.append(l)
                projs.append(lin)
                proj_index.append(gi)
    else:
        # predlayer (distill.py:100-107): one independent Linear + GELU head per distilled layer, all applied to
        # the last student hidden state (lightning.py:259-260); same seeded weight recipe per head
        for g in groups:
            layers.extend(g)
        for gi in range(len(layers)):
            lin = torch.nn.Linear(D, tcfg["encoder_embed_dim"])
            with torch.no_grad():
                lin.weight.copy_(torch.eye(D) + seeded_tensor(f"proj{gi}.weight", (D, D), seed) * 0.05)
                lin.bias.copy_(seeded_tensor(f"proj{gi}.bias", (D,), seed))
            proj_sd[f"{gi}.weight"] = lin.weight.detach().clone()
            proj_sd[f"{gi}.bias"] = lin.bias.detach().clone()
            projs.append(torch.nn.Sequential(lin, torch.nn.GELU()))
            proj_index.append(gi)
    loss_mod = ref_lightning.DistillLoss(l2_weight=l2, l1_weight=1.0, cos_weight=1.0, cos_type=cos_type)
    use_reg = lambdas is not None
    dm = ref_lightning.DistillModule(
        teacher_model=teacher, student_model=student, distill_mode=distill_mode, distill_layers=layers,
        distill_linear_projs=projs, distill_loss=loss_mod, learning_rate=2e-4, weight_decay=0.0,
        warmup_updates=15000, max_updates=50000, use_reg=use_reg, reg_learning_rate=0.02 if use_reg else None,
        target_sparsity=0.75 if use_reg else None, sparsity_warmup_updates=5000 if use_reg else None,
        tsv_dir=".", train_subset="train100", seconds_per_batch=160, num_workers=0)
    if use_reg:
        with torch.no_grad():
            dm.lambda1.fill_(lambdas[0])
            dm.lambda2.fill_(lambdas[1])
    dm.global_step = global_step
    dm.train()
    wave, ln = wave_batch(B, S, lengths=lengths)
    # capture student hiddens through a wrapper around extract_features
    cap = {}
    orig_ef = student.extract_features

    def ef(*a, **k):
        r = orig_ef(*a, **k)
        cap["h"] = [x.detach().clone() for x in r[0]]
        return r

    student.extract_features = ef
    torch.manual_seed(1234)
    with URecorder(student) as rec:
        loss = dm._step((wave, ln if lengths is not None else None), 0, "train")
    loss.backward()
    with torch.no_grad():
        th, _ = teacher.extract_features(wave, ln if lengths is not None else None)
    fx = {
        "tcfg": tcfg, "scfg": scfg, "seed": seed, "B": B, "S": S, "lengths": ln if lengths is not None else None,
        "distill_layers": layers, "proj_index": proj_index,
        "proj_recipe": "eye(D) + 0.05*seeded_tensor('proj{g}.weight'); bias seeded_tensor('proj{g}.bias')",
        "lambdas": list(lambdas) if use_reg else None, "global_step": global_step, "cos_type": cos_type, "l2": l2,
        "distill_mode": distill_mode,
        "u": rec.u, "loss": loss.detach(),
        "logged": {k: (v if torch.is_tensor(v) else torch.tensor(float(v))) for k, v in dm.logged.items()},
        "original_num_params": dm.original_num_params,
        "student_hidden_ck": [checksum(h) for h in cap["h"]],
        "teacher_hidden_ck": [checksum(h) for h in th],
        "grad_ck": {n: checksum(p.grad) for n, p in student.named_parameters() if p.grad is not None},
        "proj_grad_ck": {n: checksum(p.grad) for n, p in projs.named_parameters() if p.grad is not None},
        "log_alpha_grads": {n: p.grad.detach().clone() for n, p in student.named_parameters()
                            if n.endswith("log_alpha") and p.grad is not None},
    }
    if use_reg:
        fx["lambda_grads"] = [dm.lambda1.grad.detach().clone(), dm.lambda2.grad.detach().clone()]
    if full:
        fx["student_hiddens"] = cap["h"]
    if whole is not None:
        fx["whole_f32"] = {n: p.grad.detach().clone() for n, p in student.named_parameters()
                           if p.grad is not None and whole(n)}
    return fx


def gen_ops():
    """G1: per-op fixtures at small shapes (full tensors)."""
    torch.manual_seed(7)
    out = {}
    # HardConcrete train sample + l0 + eval mask (hardconcrete.py)
    for n_in, init_mean in [(12, 0.01), (64, 0.5), (1, 0.01)]:
        hc = HardConcrete(n_in, init_mean=init_mean)
        with torch.no_grad():
            hc.log_alpha.copy_(torch.randn(n_in) * 2.0)
        hc.train()
        with URecorder(hc) as rec:
            m = hc()
        u = rec.u[""]
        hc.eval()
        em = hc()
        out[f"hc_{n_in}"] = {"log_alpha": hc.log_alpha.detach().clone(), "u": u, "mask": m.detach().clone(),
                             "l0": hc.l0_norm().detach().clone(), "eval_mask": em.detach().clone()}
    # distill loss (lightning.py:116-139)
    s = torch.randn(2, 3, 7, 16)
    t = torch.randn(2, 3, 7, 16)
    for cos_type in ["raw", "log_sig"]:
        for w in [(0.0, 1.0, 1.0), (0.5, 1.0, 2.0)]:
            lm = ref_lightning.DistillLoss(l2_weight=w[0], l1_weight=w[1], cos_weight=w[2], cos_type=cos_type)
            si = s.clone().requires_grad_(True)
            loss, (mse, l1, cos) = lm(si, t)
            loss.backward()
            out[f"loss_{cos_type}_{w[0]}_{w[2]}"] = {
                "s": s, "t": t, "w": torch.tensor(w), "loss": loss.detach(), "mse": torch.as_tensor(mse).detach(),
                "l1": torch.as_tensor(l1).detach(), "cos": torch.as_tensor(cos).detach(), "grad": si.grad.clone()}
    # expected #params with all five pruning units, seeded log_alpha (model.py:109)
    cfg = small_cfg(3, **units_flags("conv,head,interm,attlayer,ffnlayer"))
    m, sd = seeded_model(cfg, 3)
    out["num_params"] = {"cfg": cfg, "seed": 3, "value": m.get_num_params().detach(),
                         "teacher_numel": sum(p.numel() for p in seeded_model(small_cfg(3), 3)[0].parameters())}
    # LR schedule formula (lightning.py:37-44); class itself fails on torch 2.10 (verbose kwarg)
    return out


def gen_prune():
    """G4: eval-mode prune() round trip (model.py:115-125)."""
    cfg = small_cfg(2, **units_flags("conv,head,interm,attlayer,ffnlayer"))
    m, sd = seeded_model(cfg, 5)
    g = torch.Generator()
    g.manual_seed(11)
    la = {}
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("log_alpha"):
                v = torch.randn(p.shape, generator=g) * 3.0 + (1.0 if p.numel() > 1 else 3.0)
                p.copy_(v)
                la[n] = v.clone()
    wave, _ = wave_batch(1, 16000, seed=9)
    res = m.prune()
    conv_config, use_attention, use_feed_forward, num_heads, remaining_heads, ff_interm = res
    # rebuild from the pruned config and reload, as prune.py:62-66,100-105 does
    pcfg = dict(cfg, extractor_conv_layer_config=conv_config, encoder_use_attention=use_attention,
                encoder_use_feed_forward=use_feed_forward, encoder_num_heads=num_heads,
                encoder_ff_interm_features=ff_interm, extractor_prune_conv_channels=False,
                encoder_prune_attention_heads=False, encoder_prune_attention_layer=False,
                encoder_prune_feed_forward_intermediate=False, encoder_prune_feed_forward_layer=False)
    pm = wav2vec2_model(**copy.deepcopy(pcfg))
    pm.load_state_dict(m.state_dict(), strict=True)
    pm.eval()
    with torch.no_grad():
        h, _ = pm.extract_features(wave)
    return {"cfg": cfg, "seed": 5, "log_alpha": la, "conv_config": [list(x) for x in conv_config],
            "use_attention": use_attention, "use_feed_forward": use_feed_forward, "num_heads": num_heads,
            "ff_interm_features": ff_interm, "pruned_cfg": pcfg, "state_dict_ck": {k: checksum(v) for k, v in m.state_dict().items()},
            "wave": wave, "pruned_hidden_ck": [checksum(x) for x in h]}


def gen_data():
    """G5: data-pipeline fixtures -- the reference's samplers and collate on synthetic lengths."""
    from dataset.audio_dataset import BucketizeBatchSampler, CollateFnAudio, DistributedBatchSampler  # reference
    g = torch.Generator().manual_seed(5)
    lengths = torch.randint(20000, 260000, (600,), generator=g).tolist()
    out = {"lengths": torch.tensor(lengths)}
    bs = BucketizeBatchSampler(lengths, num_buckets=50, max_token_count=900000, min_len=32000, max_len=250000,
                               shuffle=False)
    out["token_batches"] = [torch.tensor(b) for b in bs.iter_list]
    bs2 = BucketizeBatchSampler(lengths, num_buckets=20, batch_size=7, min_len=32000, max_len=250000,
                                shuffle=False, drop_last=True)
    out["size_batches"] = [torch.tensor(b) for b in bs2.iter_list]
    torch.manual_seed(11)
    bs3 = BucketizeBatchSampler(lengths, num_buckets=50, max_token_count=900000, min_len=32000, max_len=250000,
                                shuffle=True)
    out["shuffled_token_batches"] = [torch.tensor(b) for b in bs3.iter_list]
    for world in (2, 3):
        for drop in (False, True):
            for r in range(world):
                ds = DistributedBatchSampler(bs, num_replicas=world, rank=r, shuffle=True, seed=3, drop_last=drop)
                out[f"dist_w{world}_d{int(drop)}_r{r}"] = [torch.tensor(b) for b in ds.subset]
    waves = [torch.randn(1, n, generator=g) for n in (4000, 3500, 5123)]
    batch = [(w, w.shape[1]) for w in waves]
    out["collate_in"] = waves
    torch.manual_seed(13)
    out["collate_crop"] = CollateFnAudio(pad=False, rand_crop=True)(batch)
    out["collate_pad"] = CollateFnAudio(pad=True, rand_crop=False)(batch)
    return out


def gen_prenorm():
    """G6: wav2vec2-Large-style layers (pre-norm, normalize_waveform=True; run_large.sh:11 teacher
    family) on the 2-layer shape, padded batch, all five pruning units, regulariser active."""
    cfg = small_cfg(2, encoder_layer_norm_first=True, normalize_waveform=True)
    return run_step(cfg, cfg, "0.1,2", B=2, S=24000, units="conv,head,interm,attlayer,ffnlayer",
                    lambdas=(0.2, 0.1), global_step=2500, lengths=[24000, 18000], full=True)


def gen_lnext():
    """G7: layer_norm-mode extractor with conv bias (wav2vec2-Large-LV60 / HuBERT-Large family:
    LayerNorm over channels after every conv) + pre-norm layers, 2-layer shape, padded batch."""
    cfg = small_cfg(2, extractor_mode="layer_norm", extractor_conv_bias=True, encoder_layer_norm_first=True)
    return run_step(cfg, cfg, "0.1,2", B=2, S=24000, units="conv,head,interm", lambdas=(0.2, 0.1),
                    global_step=2500, lengths=[24000, 19000], full=True)


def wavlm_cfg(n_layers, remaining_heads=None, **kw):
    """WavLM config (model.py:736 wavlm_model keys): no encoder_num_heads / encoder_head_dim, total + remaining
    heads per layer, relative-position buckets."""
    c = small_cfg(n_layers)
    del c["encoder_num_heads"], c["encoder_head_dim"]
    c.update(encoder_total_num_heads=[12] * n_layers,
             encoder_remaining_heads=remaining_heads or [list(range(12))] * n_layers,
             encoder_num_buckets=32, encoder_max_distance=40)
    c.update(kw)
    return c


def gen_wavlm():
    """G8: WavLM layers (WavLMSelfAttention, components.py:486-659: bucketed relative-position bias from layer
    0's embedding shared by every layer, GRU-style gate per layer) on the 2-layer shape, padded batch, layer 1
    with 9 of 12 heads remaining, regulariser active.  num_buckets 32 / max_distance 40 so T = 74 frames reach
    both the log-spaced buckets and the num_buckets-1 cap."""
    cfg = wavlm_cfg(2, remaining_heads=[list(range(12)), [0, 1, 3, 4, 6, 7, 8, 10, 11]])
    fx = run_step(cfg, cfg, "0.1,2", B=2, S=24000, units="conv,head,interm", lambdas=(0.2, 0.1),
                  global_step=2500, lengths=[24000, 19000], full=True)
    m, _ = seeded_model(dict(cfg, **units_flags("conv,head,interm")), 0)
    fx["sd_schema"] = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    fx["num_params_init"] = float(m.get_num_params())
    # the bucket table of the reference for T = 74 and a long T (integer index data)
    from wav2vec2.components import WavLMSelfAttention
    att = WavLMSelfAttention(64, 1, has_relative_attention_bias=True, num_buckets=320, max_distance=800)
    fx["bucket_320_800_T1000"] = att._relative_positions_bucket(
        torch.arange(1000)[None, :] - torch.arange(1000)[:, None], bidirectional=True)[0].clone()
    att = WavLMSelfAttention(64, 1, has_relative_attention_bias=True, num_buckets=32, max_distance=40)
    fx["bucket_32_40_T200"] = att._relative_positions_bucket(
        torch.arange(200)[None, :] - torch.arange(200)[:, None], bidirectional=True)[0].clone()
    return fx


def gen_wavlm_prune():
    """G9: eval-mode prune() of a WavLM model (WavLMSelfAttention.prune, components.py:661-693: remaining_heads
    instead of num_heads) with all five units, rebuilt from the pruned config (prune.py:25-39), plus the pruned
    model's hidden states on a padded batch."""
    cfg = wavlm_cfg(2, **units_flags("conv,head,interm,attlayer,ffnlayer"))
    m, sd = seeded_model(cfg, 5)
    g = torch.Generator()
    g.manual_seed(12)
    la = {}
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("log_alpha"):
                v = torch.randn(p.shape, generator=g) * 3.0 + (1.0 if p.numel() > 1 else 3.0)
                p.copy_(v)
                la[n] = v.clone()
    wave, ln = wave_batch(2, 24000, seed=9, lengths=[24000, 20000])
    conv_config, use_attention, use_feed_forward, num_heads, remaining_heads, ff_interm = m.prune()
    pcfg = dict(cfg, extractor_conv_layer_config=conv_config, encoder_use_attention=use_attention,
                encoder_use_feed_forward=use_feed_forward, encoder_remaining_heads=remaining_heads,
                encoder_ff_interm_features=ff_interm, extractor_prune_conv_channels=False,
                encoder_prune_attention_heads=False, encoder_prune_attention_layer=False,
                encoder_prune_feed_forward_intermediate=False, encoder_prune_feed_forward_layer=False)
    pm = wav2vec2_model(**copy.deepcopy(pcfg))
    pm.load_state_dict(m.state_dict(), strict=True)
    pm.eval()
    with torch.no_grad():
        h, _ = pm.extract_features(wave, ln)
    return {"cfg": cfg, "seed": 5, "log_alpha": la, "conv_config": [list(x) for x in conv_config],
            "use_attention": use_attention, "use_feed_forward": use_feed_forward, "remaining_heads": remaining_heads,
            "num_heads": num_heads, "ff_interm_features": ff_interm, "pruned_cfg": pcfg,
            "state_dict_ck": {k: checksum(v) for k, v in m.state_dict().items()},
            "wave": wave, "lengths": ln, "pruned_hiddens": [x.clone() for x in h]}


def large_cfg(n_layers, **kw):
    """wav2vec2-Large dimensions (convert_wav2vec2_large_from_fairseq.py:19-40; run_large.sh:11 teacher): D 1024,
    16 heads, FFN 4096, pre-norm, normalize_waveform, group_norm extractor; n_layers of the 24, dropout 0."""
    c = small_cfg(n_layers, encoder_embed_dim=1024, encoder_num_heads=[16] * n_layers,
                  encoder_ff_interm_features=[4096] * n_layers, encoder_layer_norm_first=True, normalize_waveform=True)
    c.update(kw)
    return c


def gen_base12():
    """G3: full Base 12 layers, 1 x 10 s, distill layers 0.4,8,12 (checksums only)."""
    return run_step(no_dropout(HUBERT_BASE_CONFIG), no_dropout(HUBERT_BASE_CONFIG), "0.4,8,12", B=1, S=160000,
                    units="conv,head,interm", lambdas=(0.0, 0.0), global_step=5000)


def _g14_whole(n):
    """The parameters g14 stores whole gradients of: the last two encoder layers' attention projections, the last
    layer's feed-forward and LayerNorms, and the conv frontend's first and last two layers + GroupNorm and the
    feature projection (the rest of the frontend is ~3 M more parameters; every other gradient keeps its 64-sample
    checksum)."""
    if "log_alpha" in n:
        return False
    if n.startswith("encoder.transformer.layers.11."):
        return True
    if n.startswith("encoder.transformer.layers.10.attention.") and "hard_concrete" not in n:
        return True
    return n.startswith(("feature_extractor.conv_layers.0.", "feature_extractor.conv_layers.5.",
                         "feature_extractor.conv_layers.6.", "encoder.feature_projection."))


def gen_base12_whole():
    """G14: G3's configuration (full Base 12 layers, 1 x 10 s, distill layers 0.4,8,12) with whole gradients of the
    _g14_whole parameters (bf16 values + fp32 norms + bf16-emulation sensitivity per tensor)."""
    return run_step(no_dropout(HUBERT_BASE_CONFIG), no_dropout(HUBERT_BASE_CONFIG), "0.4,8,12", B=1, S=160000,
                    units="conv,head,interm", lambdas=(0.0, 0.0), global_step=5000, whole=_g14_whole)


def gen_large():
    """G10: Large dimensions, 2 layers, one utterance at lightning.py:313's max_len 250000 samples (T = 781) and a
    shorter padded one, all of conv,head,interm, regulariser active (checksums only: full hiddens are 6 MB each)."""
    cfg = large_cfg(2)
    return run_step(cfg, cfg, "0.1,2", B=2, S=250000, units="conv,head,interm", lambdas=(0.2, 0.1),
                    global_step=2500, lengths=[250000, 201234])


def gen_large_ln():
    """G11: HuBERT-Large family (convert_hubert_large_from_fairseq.py:19-40: layer_norm extractor) at Large
    dimensions, 2 layers, 1 x 4 s, all five units."""
    cfg = large_cfg(2, extractor_mode="layer_norm")
    return run_step(cfg, cfg, "0.1,2", B=1, S=64000, units="conv,head,interm,attlayer,ffnlayer",
                    lambdas=(0.3, -0.1), global_step=6000)


def gen_large24():
    """G13: the whole wav2vec2-Large teacher depth of run_large.sh (24 pre-norm layers, D 1024, normalize_waveform,
    distill layers 0.4,8,12,16,20,24 = run_large.sh:13), 1 x 2 s, conv,head,interm, regulariser active (checksums)."""
    cfg = large_cfg(24)
    return run_step(cfg, cfg, "0.4,8,12,16,20,24", B=1, S=32000, units="conv,head,interm", lambdas=(0.2, 0.1),
                    global_step=5000)


def _g15_whole(n):
    """g15's whole-gradient set: layer 0's attention projections, every parameter of the last (4th) layer, the
    transformer's closing LayerNorm (pre-norm), conv0 / conv5 / conv6 + GroupNorm and the feature projection."""
    if "log_alpha" in n or "hard_concrete" in n:
        return False
    if n.startswith(("encoder.transformer.layers.3.", "encoder.transformer.layer_norm.")):
        return True
    if n.startswith("encoder.transformer.layers.0.attention."):
        return True
    return n.startswith(("feature_extractor.conv_layers.0.", "feature_extractor.conv_layers.5.",
                         "feature_extractor.conv_layers.6.", "encoder.feature_projection."))


def gen_large_whole():
    """G15: pre-norm Large width (D 1024, 16 heads, FFN 4096, normalize_waveform, group_norm extractor), 4 layers, one
    utterance at lightning.py:313's max_len 250000 samples (T = 781), distill layers 0.2,4, conv,head,interm with the
    regulariser active; whole gradients of the _g15_whole parameters (bf16 values + fp32 norms + bf16-emulation
    sensitivity per tensor), checked like g14 (components.py:848-850 pre-norm, model.py:96-103)."""
    cfg = large_cfg(4)
    return run_step(cfg, cfg, "0.2,4", B=1, S=250000, units="conv,head,interm", lambdas=(0.2, 0.1),
                    global_step=5000, whole=_g15_whole)


def gen_predlayer():
    """G12: predlayer distill mode (distill.py:100-107, lightning.py:259-260) on the 2-layer Base shape, three
    heads (distill layers 0,1,2) on the last hidden state, padded batch, regulariser active."""
    c = small_cfg(2)
    return run_step(c, c, "0,1,2", B=2, S=24000, units="conv,head,interm", lambdas=(0.2, 0.1), global_step=2500,
                    lengths=[24000, 21000], full=True, distill_mode="predlayer")


def main():
    only = [a[len("--only="):] for a in sys.argv[1:] if a.startswith("--only=")]
    extra = {"g10_large.pt": gen_large, "g11_large_lnext.pt": gen_large_ln, "g12_predlayer.pt": gen_predlayer,
             "g3_base12.pt": gen_base12, "g13_large24.pt": gen_large24, "g14_base12_whole.pt": gen_base12_whole,
             "g15_large4_whole.pt": gen_large_whole}
    if only:
        OUT.mkdir(parents=True, exist_ok=True)
        torch.set_num_threads(8)
        for name in only:
            fx = extra[name]()
            torch.save(fx, OUT / name)
            print(name, "done", fx["loss"].item() if "loss" in fx else "")
        return
    OUT.mkdir(parents=True, exist_ok=True)
    torch.set_num_threads(8)
    if "--only-wavlm-prune" in sys.argv:
        torch.save(gen_wavlm_prune(), OUT / "g9_wavlm_prune.pt")
        print("g9 done")
        return
    if "--only-wavlm" in sys.argv:
        torch.save(gen_wavlm(), OUT / "g8_wavlm.pt")
        print("g8 done")
        return
    if "--only-lnext" in sys.argv:
        torch.save(gen_lnext(), OUT / "g7_lnext.pt")
        print("g7 done")
        return
    if "--only-data" in sys.argv:
        torch.save(gen_data(), OUT / "g5_data.pt")
        print("g5 done")
        return
    if "--only-prenorm" in sys.argv:
        torch.save(gen_prenorm(), OUT / "g6_prenorm_normwave.pt")
        print("g6 done")
        return
    torch.save(gen_data(), OUT / "g5_data.pt")
    print("g5 done")
    torch.save(gen_prenorm(), OUT / "g6_prenorm_normwave.pt")
    print("g6 done")
    torch.save(gen_ops(), OUT / "g1_ops.pt")
    print("g1 done")
    # G2: 2-layer smoke step (BASELINE config 1 shape-reduced to 2 s), units conv,head,interm, reg active
    g2 = run_step(small_cfg(2), small_cfg(2), "0.1,2", B=2, S=32000, units="conv,head,interm",
                  lambdas=(0.3, 0.2), global_step=1000, full=True)
    torch.save(g2, OUT / "g2_smoke_step.pt")
    print("g2 done", g2["loss"].item())
    # G2b: all five units, padded batch (lengths), log_sig cosine + l2
    g2b = run_step(small_cfg(2), small_cfg(2), "0.1,2", B=2, S=24000, units="conv,head,interm,attlayer,ffnlayer",
                   lambdas=(-0.1, 0.05), global_step=7000, lengths=[24000, 17000], cos_type="log_sig", l2=0.5)
    torch.save(g2b, OUT / "g2b_all_units_padded.pt")
    print("g2b done", g2b["loss"].item())
    # G3: full Base 12 layers, 1 x 10 s, distill layers 0.4,8,12 (checksums only)
    g3 = gen_base12()
    torch.save(g3, OUT / "g3_base12.pt")
    print("g3 done", g3["loss"].item())
    torch.save(gen_prune(), OUT / "g4_prune.pt")
    print("g4 done")


if __name__ == "__main__":
    main()
