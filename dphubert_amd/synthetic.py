"""Seeded synthetic weights and batches.

There is no network in this environment, so no pretrained HuBERT checkpoint is
available.  Every parity fixture, test and benchmark therefore uses weights made
by :func:`seeded_tensor`, a pure function of ``(seed, parameter name, shape)``:
the golden generator (``tools/gen_golden.py``) fills the *reference* model with
it, and the tests fill this package's model with it, so both see bit-identical
fp32 parameters without shipping a checkpoint.

Magnitudes mimic a trained model closely enough that activations stay O(1)
through 12 post-norm layers (fan-in scaled weights, LN gains near 1).
HardConcrete ``log_alpha`` follows the reference init
(wav2vec2/hardconcrete.py:70-74: ``normal(log(1-m) - log(m), 0.01)``).
"""

import math
import zlib
from typing import Dict, Iterable, Tuple

import torch

__all__ = [
    "HUBERT_BASE_CONFIG",
    "HUBERT_LARGE_CONFIG",
    "WAV2VEC2_LARGE_CONFIG",
    "pruned_student",
    "seeded_tensor",
    "seeded_state_dict",
    "synthetic_batch",
]

# default config of HuBERT Base, as written by convert_hubert_from_hf.py:18-44
HUBERT_BASE_CONFIG = dict(
    extractor_mode="group_norm",
    extractor_conv_layer_config=[(512, 10, 5)] + [(512, 3, 2)] * 4 + [(512, 2, 2)] * 2,
    extractor_conv_bias=False,
    encoder_embed_dim=768,
    encoder_projection_dropout=0.1,
    encoder_pos_conv_kernel=128,
    encoder_pos_conv_groups=16,
    encoder_num_layers=12,
    encoder_use_attention=[True] * 12,
    encoder_use_feed_forward=[True] * 12,
    encoder_num_heads=[12] * 12,
    encoder_head_dim=64,
    encoder_attention_dropout=0.1,
    encoder_ff_interm_features=[3072] * 12,
    encoder_ff_interm_dropout=0.0,
    encoder_dropout=0.1,
    encoder_layer_norm_first=False,
    encoder_layer_drop=0.05,
    aux_num_out=None,
    normalize_waveform=False,
    extractor_prune_conv_channels=False,
    encoder_prune_attention_heads=False,
    encoder_prune_attention_layer=False,
    encoder_prune_feed_forward_intermediate=False,
    encoder_prune_feed_forward_layer=False,
)

# WavLM Base (model.py:865-914 wavlm_base; convert_wavlm_from_hf.py config layout: total + remaining heads per layer,
# 320 relative-position buckets up to 800 frames)
WAVLM_BASE_CONFIG = {k: v for k, v in HUBERT_BASE_CONFIG.items() if k not in ("encoder_num_heads", "encoder_head_dim")}
WAVLM_BASE_CONFIG.update(encoder_total_num_heads=[12] * 12, encoder_remaining_heads=[list(range(12))] * 12,
                         encoder_num_buckets=320, encoder_max_distance=800)

# wav2vec2-large teacher of run_large.sh (convert_wav2vec2_large_from_fairseq.py:19-40)
HUBERT_LARGE_CONFIG = dict(
    HUBERT_BASE_CONFIG,
    extractor_mode="layer_norm",
    extractor_conv_bias=True,
    encoder_embed_dim=1024,
    encoder_projection_dropout=0.0,
    encoder_num_layers=24,
    encoder_use_attention=[True] * 24,
    encoder_use_feed_forward=[True] * 24,
    encoder_num_heads=[16] * 24,
    encoder_attention_dropout=0.0,
    encoder_ff_interm_features=[4096] * 24,
    encoder_dropout=0.0,
    encoder_layer_norm_first=True,
    encoder_layer_drop=0.0,
    normalize_waveform=True,
)


# the wav2vec2-Large teacher run_large.sh:11 distils (convert_wav2vec2_large_from_fairseq.py:19-40): group_norm
# extractor without conv bias, 24 pre-norm layers of width 1024 / 16 heads / FFN 4096, normalize_waveform
WAV2VEC2_LARGE_CONFIG = dict(
    HUBERT_BASE_CONFIG,
    encoder_embed_dim=1024,
    encoder_num_layers=24,
    encoder_use_attention=[True] * 24,
    encoder_use_feed_forward=[True] * 24,
    encoder_num_heads=[16] * 24,
    encoder_ff_interm_features=[4096] * 24,
    encoder_layer_norm_first=True,
    normalize_waveform=True,
)

# DPHuBERT's published parameter count (README.md:110-111): the student final_distill.py trains
DPHUBERT_PARAMS = 23_585_946


def _gen(seed: int, name: str) -> torch.Generator:
    g = torch.Generator()
    g.manual_seed((int(seed) * 1000003 + zlib.crc32(name.encode())) % (2**63 - 1))
    return g


def seeded_tensor(name: str, shape: Tuple[int, ...], seed: int = 0) -> torch.Tensor:
    """Deterministic fp32 value for parameter ``name`` of ``shape``."""
    shape = tuple(int(s) for s in shape)
    g = _gen(seed, name)
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "dummy_weight":
        return torch.ones(shape)
    if leaf == "log_alpha":
        # reference init: interm units use init_mean=0.5, everything else 0.01
        # (components.py:90,370,375,715-722)
        init_mean = 0.5 if "hard_concrete_for_intermediate" in name else 0.01
        mean = math.log(1 - init_mean) - math.log(init_mean)
        return torch.randn(shape, generator=g) * 0.01 + mean
    if leaf == "weight_g":
        return 2.4 * (1.0 + 0.1 * torch.randn(shape, generator=g))
    if leaf == "weight_v":
        return torch.randn(shape, generator=g)
    is_norm = ("layer_norm" in name) or ("final_layer_norm" in name)
    if leaf == "weight" and is_norm:
        return 1.0 + 0.1 * torch.randn(shape, generator=g)
    if leaf == "bias":
        return (0.1 if is_norm else 0.02) * torch.randn(shape, generator=g)
    if leaf == "weight":
        fan_in = 1
        for s in shape[1:]:
            fan_in *= s
        return torch.randn(shape, generator=g) / math.sqrt(max(fan_in, 1))
    if leaf == "gru_rel_pos_const":
        # WavLM gate constant: reference init is ones (components.py:541); perturbed so its grad is non-trivial
        return 1.0 + 0.1 * torch.randn(shape, generator=g)
    if leaf in ("lambda1", "lambda2"):
        return torch.zeros(shape)
    return 0.02 * torch.randn(shape, generator=g)


def seeded_state_dict(shapes: Iterable[Tuple[str, Tuple[int, ...]]], seed: int = 0) -> Dict[str, torch.Tensor]:
    return {n: seeded_tensor(n, s, seed) for n, s in shapes}


def synthetic_batch(batch: int, samples: int = 160000, seed: int = 2022):
    """``0.1*randn(B,S)`` waveforms + full lengths."""
    g = torch.Generator()
    g.manual_seed(seed)
    wave = 0.1 * torch.randn(batch, samples, generator=g)
    lengths = torch.full((batch,), samples, dtype=torch.int64)
    return wave, lengths


def _param_count(config: dict) -> int:
    from .wav2vec2.model import wav2vec2_model
    with torch.device("meta"):
        m = wav2vec2_model(**config)
    return sum(p.numel() for p in m.parameters())


def pruned_student(config: dict, target_params: int = DPHUBERT_PARAMS, seed: int = 0):
    """A final_distill.py student (final_distill.py:61-65): the reference's own prune() (model.py:115-125) applied to
    a conv,head,interm student whose HardConcrete logits keep a seeded, per-layer ragged number of conv channels,
    heads and FFN units, scaled so that the pruned model has ~``target_params`` parameters (23.59 M: DPHuBERT,
    README.md:110).  Returns (pruned config, pruned state_dict); the weights are the seeded teacher weights that
    survive the pruning (the student is initialised from the teacher, run.sh:20).
    """
    import copy
    from .wav2vec2.model import wav2vec2_model
    units = dict(copy.deepcopy(config), extractor_prune_conv_channels=True, encoder_prune_attention_heads=True,
                 encoder_prune_feed_forward_intermediate=True)
    g = torch.Generator().manual_seed(1000 + seed)
    n_layers = config["encoder_num_layers"]
    convs = [c for c, _, _ in config["extractor_conv_layer_config"]]
    heads = list(config["encoder_num_heads"])
    ffs = list(config["encoder_ff_interm_features"])
    jc = (0.75 + 0.5 * torch.rand(len(convs), generator=g)).tolist()
    jh = (0.75 + 0.5 * torch.rand(n_layers, generator=g)).tolist()
    jf = (0.75 + 0.5 * torch.rand(n_layers, generator=g)).tolist()

    def arch(r):
        kc = [max(8, min(c, round(c * r * j))) for c, j in zip(convs, jc)]
        kh = [max(1, min(h, round(h * r * j))) for h, j in zip(heads, jh)]
        kf = [max(8, min(f, round(f * r * j))) for f, j in zip(ffs, jf)]
        return kc, kh, kf

    def count(r):
        kc, kh, kf = arch(r)
        c = copy.deepcopy(config)
        c["extractor_conv_layer_config"] = [(k, kk, ss) for k, (_, kk, ss) in zip(kc, config["extractor_conv_layer_config"])]
        c["encoder_num_heads"] = kh
        c["encoder_ff_interm_features"] = kf
        return _param_count(c)

    lo, hi = 0.02, 1.0
    for _ in range(30):
        mid = 0.5 * (lo + hi)
        if count(mid) > target_params:
            hi = mid
        else:
            lo = mid
    kc, kh, kf = arch(lo if abs(count(lo) - target_params) <= abs(count(hi) - target_params) else hi)
    model = wav2vec2_model(**copy.deepcopy(units))
    model.load_state_dict(seeded_state_dict([(k, tuple(v.shape)) for k, v in model.state_dict().items()], seed))
    keep = {}
    fe = model.feature_extractor.conv_layers
    for i, k in enumerate(kc):
        keep[fe[i].hard_concrete] = k
    for l, layer in enumerate(model.encoder.transformer.layers):
        keep[layer.attention.hard_concrete_for_heads] = kh[l]
        keep[layer.feed_forward.hard_concrete_for_intermediate] = kf[l]
    with torch.no_grad():
        for hc, k in keep.items():
            la = torch.full((hc.n_in,), -12.0)
            la[torch.randperm(hc.n_in, generator=g)[:k]] = 12.0
            hc.log_alpha.copy_(la)
    model.eval()
    conv_config, use_attention, use_feed_forward, num_heads, remaining_heads, ff_interm = model.prune()
    pruned = copy.deepcopy(config)
    pruned.update({"extractor_conv_layer_config": conv_config, "encoder_use_attention": use_attention,
                   "encoder_use_feed_forward": use_feed_forward, "encoder_num_heads": num_heads,
                   "encoder_ff_interm_features": ff_interm})
    return pruned, {k: v.detach().clone() for k, v in model.state_dict().items()}
