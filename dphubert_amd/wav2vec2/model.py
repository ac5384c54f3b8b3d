"""Speech SSL model with pruning units (drop-in for wav2vec2/model.py of the reference).

``wav2vec2_model(**config)`` accepts the reference's checkpoint config dict
(convert_hubert_from_hf.py:18-44 + the five ``*_prune_*`` flags,
model.py:181-361) and builds a model with the same state_dict schema.
``extract_features`` / ``get_num_params`` / ``prune`` keep their signatures and
meaning; the computation runs on gfx950 HIP kernels (``dphubert_amd.ops``).
"""

from typing import List, Optional, Tuple

import torch
import torch.nn.functional as F
from torch import Tensor
from torch.nn import Module

from .. import ops
from . import components
from .components import Poly, _PolyCtx


class Wav2Vec2Model(Module):
    def __init__(self, normalize_waveform: bool, feature_extractor: Module, encoder: Module,
                 aux: Optional[Module] = None):
        super().__init__()
        self.normalize_waveform = normalize_waveform
        self.feature_extractor = feature_extractor
        self.encoder = encoder
        self.aux = aux
        self._np_table = None
        self._np_key = None

    def _normalize(self, waveforms, lengths):
        """model.py:96-103: per-utterance LayerNorm over each waveform's valid samples (HIP kernel),
        zero padding after; like the reference's pad_sequence, the batch is cut to max(lengths)."""
        if not waveforms.is_cuda:
            raise ValueError("normalize_waveform runs on the HIP path only: pass a device tensor")
        x = waveforms.contiguous().float()
        B, S = x.shape
        ln = lengths.to(x.device, torch.int64).contiguous() if lengths is not None else None
        y = torch.empty_like(x)
        ops.call("dph_wave_layernorm", ops.ptr(x), ops.ptr(ln), B, S, 1e-5, ops.ptr(y), ops._s())
        if ln is not None:
            lmax = int(ln.max())
            if lmax < S:
                y = y[:, :lmax].contiguous()
        return y

    def extract_features(self, waveforms: Tensor, lengths: Optional[Tensor] = None,
                         num_layers: Optional[int] = None) -> Tuple[List[Tensor], Optional[Tensor]]:
        """model.py:57-107.  Returns the N+1 hidden states (B, T, D) (bf16) and the frame lengths."""
        if self.normalize_waveform:
            waveforms = self._normalize(waveforms, lengths)
        x, lengths = self.feature_extractor(waveforms, lengths)
        x = self.encoder.extract_features(x, lengths, num_layers)
        return x, lengths

    # ---- expected size ----------------------------------------------------
    def _num_params_poly(self):
        ctx = _PolyCtx()
        fe_poly, in_feat = self.feature_extractor.poly(ctx)
        total = fe_poly + self.encoder.poly(ctx, in_feat)
        return total, ctx.mods

    def get_num_params(self):
        """Differentiable expected parameter count (model.py:109-113) as a 0-d device tensor."""
        key = tuple(id(m) for m in self.modules())
        if self._np_key != key:
            poly, mods = self._num_params_poly()
            terms = [(c, k) for k, c in poly.t.items() if k and c != 0.0]
            constant = poly.t.get((), 0.0)
            dev = next(self.parameters()).device
            self._np_table = ops.ExpectedParamsTable(terms, constant, [m.n_in for m in mods], dev)
            self._np_mods = mods
            self._np_key = key
        las = [m.log_alpha for m in self._np_mods]
        if not las:
            return torch.tensor(float(self._np_table.constant), device=next(self.parameters()).device)
        return ops.ExpectedParamsFn.apply(self._np_table, *las)

    def prune(self):
        """Eval-mode structural pruning (model.py:115-125)."""
        self.eval()
        conv_config, conv_out_index = self.feature_extractor.prune()
        transformer_config = self.encoder.prune(conv_out_index)
        use_attention = transformer_config["use_attention"]
        use_feed_forward = transformer_config["use_feed_forward"]
        num_heads = transformer_config["num_heads"]
        remaining_heads = transformer_config["remaining_heads"]
        ff_interm_features = transformer_config["ff_interm_features"]
        self._np_key = None
        return conv_config, use_attention, use_feed_forward, num_heads, remaining_heads, ff_interm_features

    def forward(self, waveforms: Tensor, lengths: Optional[Tensor] = None) -> Tuple[Tensor, Optional[Tensor]]:
        """model.py:127-169."""
        if self.normalize_waveform:
            waveforms = self._normalize(waveforms, lengths)
        x, lengths = self.feature_extractor(waveforms, lengths)
        x = self.encoder(x, lengths)
        if self.aux is not None:
            x = self.aux(x.float())
        return x, lengths


def wav2vec2_model(**configs) -> Wav2Vec2Model:
    """Wraps the original wav2vec2_model (model.py:172-178)."""
    if "encoder_remaining_heads" in configs:
        return wavlm_model(**configs)
    return wav2vec2_model_original(**configs)


def wavlm_model(
    extractor_mode: str,
    extractor_conv_layer_config: Optional[List[Tuple[int, int, int]]],
    extractor_conv_bias: bool,
    encoder_embed_dim: int,
    encoder_projection_dropout: float,
    encoder_pos_conv_kernel: int,
    encoder_pos_conv_groups: int,
    encoder_num_layers: int,
    encoder_use_attention: List[bool],
    encoder_use_feed_forward: List[bool],
    encoder_total_num_heads: List[int],
    encoder_remaining_heads: List[List[int]],
    encoder_num_buckets: int,
    encoder_max_distance: int,
    encoder_attention_dropout: float,
    encoder_ff_interm_features: List[int],
    encoder_ff_interm_dropout: float,
    encoder_dropout: float,
    encoder_layer_norm_first: bool,
    encoder_layer_drop: float,
    aux_num_out: Optional[int],
    normalize_waveform: bool,
    extractor_prune_conv_channels: bool = False,
    encoder_prune_attention_heads: bool = False,
    encoder_prune_attention_layer: bool = False,
    encoder_prune_feed_forward_intermediate: bool = False,
    encoder_prune_feed_forward_layer: bool = False,
) -> Wav2Vec2Model:
    """model.py:736-862 (same arguments, same defaults): WavLM = wav2vec2 frontend + encoder with
    WavLMSelfAttention."""
    if extractor_conv_layer_config is None:
        extractor_conv_layer_config = [(512, 10, 5)] + [(512, 3, 2)] * 4 + [(512, 2, 2)] * 2
    extractor_conv_layer_config = [tuple(c) for c in extractor_conv_layer_config]
    feature_extractor = components._get_feature_extractor(
        extractor_mode, extractor_conv_layer_config, extractor_conv_bias,
        prune_conv_channels=extractor_prune_conv_channels)
    encoder = components._get_wavlm_encoder(
        in_features=extractor_conv_layer_config[-1][0], embed_dim=encoder_embed_dim,
        dropout_input=encoder_projection_dropout, pos_conv_kernel=encoder_pos_conv_kernel,
        pos_conv_groups=encoder_pos_conv_groups, num_layers=encoder_num_layers, use_attention=encoder_use_attention,
        use_feed_forward=encoder_use_feed_forward, total_num_heads=encoder_total_num_heads,
        remaining_heads=encoder_remaining_heads, num_buckets=encoder_num_buckets, max_distance=encoder_max_distance,
        attention_dropout=encoder_attention_dropout, ff_interm_features=encoder_ff_interm_features,
        ff_interm_dropout=encoder_ff_interm_dropout, dropout=encoder_dropout,
        layer_norm_first=encoder_layer_norm_first, layer_drop=encoder_layer_drop,
        prune_attention_heads=encoder_prune_attention_heads, prune_attention_layer=encoder_prune_attention_layer,
        prune_feed_forward_intermediate=encoder_prune_feed_forward_intermediate,
        prune_feed_forward_layer=encoder_prune_feed_forward_layer)
    aux = None
    if aux_num_out is not None:
        aux = torch.nn.Linear(in_features=encoder_embed_dim, out_features=aux_num_out)
    return Wav2Vec2Model(normalize_waveform, feature_extractor, encoder, aux)


def wav2vec2_model_original(
    extractor_mode: str,
    extractor_conv_layer_config: Optional[List[Tuple[int, int, int]]],
    extractor_conv_bias: bool,
    encoder_embed_dim: int,
    encoder_projection_dropout: float,
    encoder_pos_conv_kernel: int,
    encoder_pos_conv_groups: int,
    encoder_num_layers: int,
    encoder_use_attention: List[bool],
    encoder_use_feed_forward: List[bool],
    encoder_num_heads: List[int],
    encoder_head_dim: int,
    encoder_attention_dropout: float,
    encoder_ff_interm_features: List[int],
    encoder_ff_interm_dropout: float,
    encoder_dropout: float,
    encoder_layer_norm_first: bool,
    encoder_layer_drop: float,
    aux_num_out: Optional[int],
    normalize_waveform: bool,
    extractor_prune_conv_channels: bool = False,
    encoder_prune_attention_heads: bool = False,
    encoder_prune_attention_layer: bool = False,
    encoder_prune_feed_forward_intermediate: bool = False,
    encoder_prune_feed_forward_layer: bool = False,
) -> Wav2Vec2Model:
    """model.py:181-361 (same arguments, same defaults)."""
    if extractor_conv_layer_config is None:
        extractor_conv_layer_config = [(512, 10, 5)] + [(512, 3, 2)] * 4 + [(512, 2, 2)] * 2
    extractor_conv_layer_config = [tuple(c) for c in extractor_conv_layer_config]
    feature_extractor = components._get_feature_extractor(
        extractor_mode, extractor_conv_layer_config, extractor_conv_bias,
        prune_conv_channels=extractor_prune_conv_channels)
    encoder = components._get_encoder(
        in_features=extractor_conv_layer_config[-1][0], embed_dim=encoder_embed_dim,
        dropout_input=encoder_projection_dropout, pos_conv_kernel=encoder_pos_conv_kernel,
        pos_conv_groups=encoder_pos_conv_groups, num_layers=encoder_num_layers, use_attention=encoder_use_attention,
        use_feed_forward=encoder_use_feed_forward, num_heads=encoder_num_heads, head_dim=encoder_head_dim,
        attention_dropout=encoder_attention_dropout, ff_interm_features=encoder_ff_interm_features,
        ff_interm_dropout=encoder_ff_interm_dropout, dropout=encoder_dropout,
        layer_norm_first=encoder_layer_norm_first, layer_drop=encoder_layer_drop,
        prune_attention_heads=encoder_prune_attention_heads, prune_attention_layer=encoder_prune_attention_layer,
        prune_feed_forward_intermediate=encoder_prune_feed_forward_intermediate,
        prune_feed_forward_layer=encoder_prune_feed_forward_layer)
    aux = None
    if aux_num_out is not None:
        aux = torch.nn.Linear(in_features=encoder_embed_dim, out_features=aux_num_out)
    return Wav2Vec2Model(normalize_waveform, feature_extractor, encoder, aux)
