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
        self._np_mods = None
        self._bank = None
        self._bank_num = None      # (expected #params of the last batched gate launch, log_alpha versions)
        self._lmax_hint = None     # crop length of the last eager _normalize (used while a HIP graph is captured)

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
            # pad_sequence cuts the batch to max(lengths); that needs the value on the host.  While a HIP graph
            # is being captured no device->host read is allowed: the crop of the preceding eager step (same
            # batch shape) is reused -- crop-to-min collation gives lmax == S anyway
            if torch.cuda.is_current_stream_capturing():
                if self._lmax_hint is None or self._lmax_hint[0] != S:
                    raise RuntimeError("normalize_waveform under HIP-graph capture needs an eager step of the same "
                                       "batch shape first (its crop length is reused)")
                lmax = self._lmax_hint[1]
            else:
                lmax = int(ln.max())
                self._lmax_hint = (S, lmax)
            if lmax < S:
                y = y[:, :lmax].contiguous()
        return y

    def _sample_gates(self):
        """Training mode: sample every HardConcrete gate of the model in ONE launch (and its expected #params)
        before the forward; each gate's forward() then hands out its slice."""
        self._bank_num = None
        if not self.training or not next(self.parameters()).is_cuda:
            return
        self._ensure_table()
        mods = self._np_mods
        if not mods:
            return
        if self._bank is None or self._bank.mods != mods:
            self._bank = ops.HardConcreteBank(mods, self._np_table)
        las = [m.log_alpha for m in mods]
        outs = ops.HardConcreteBankFn.apply(self._bank, *las)
        for m, mask in zip(mods, outs[:-1]):
            m._bank_mask = mask
        self._bank_num = (outs[-1], tuple((id(la), la._version) for la in las))

    def _drop_gates(self):
        for m in (self._np_mods or []) if self._bank is not None else []:
            m._bank_mask = None

    def extract_features(self, waveforms: Tensor, lengths: Optional[Tensor] = None,
                         num_layers: Optional[int] = None) -> Tuple[List[Tensor], Optional[Tensor]]:
        """model.py:57-107.  Returns the N+1 hidden states (B, T, D) and the frame lengths: bf16, and fp32 for the
        layers of a pre-norm encoder (its residual stream, ops.EncoderLayerFn._forward_pre)."""
        if self.normalize_waveform:
            waveforms = self._normalize(waveforms, lengths)
        self._sample_gates()
        try:
            x, lengths = self.feature_extractor(waveforms, lengths)
            x = self.encoder.extract_features(x, lengths, num_layers)
        finally:
            self._drop_gates()
        return x, lengths

    # ---- expected size ----------------------------------------------------
    def _num_params_poly(self):
        ctx = _PolyCtx()
        fe_poly, in_feat = self.feature_extractor.poly(ctx)
        total = fe_poly + self.encoder.poly(ctx, in_feat)
        return total, ctx.mods

    def _ensure_table(self):
        key = tuple(id(m) for m in self.modules()) + (next(self.parameters()).device,)
        if self._np_key != key:
            poly, mods = self._num_params_poly()
            terms = [(c, k) for k, c in poly.t.items() if k and c != 0.0]
            constant = poly.t.get((), 0.0)
            dev = next(self.parameters()).device
            self._np_table = ops.ExpectedParamsTable(terms, constant, [m.n_in for m in mods], dev)
            self._np_mods = mods
            self._np_key = key
            self._bank = None

    def get_num_params(self):
        """Differentiable expected parameter count (model.py:109-113) as a 0-d device tensor.  In training mode
        it is the value computed with this step's batched gate launch (one backward node for both gradients of
        every log_alpha), while the log_alphas are unchanged since."""
        self._ensure_table()
        las = [m.log_alpha for m in self._np_mods]
        if self._bank_num is not None:
            num, key = self._bank_num
            self._bank_num = None
            if key == tuple((id(la), la._version) for la in las):
                return num
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
        self._bank = None
        self._bank_num = None
        return conv_config, use_attention, use_feed_forward, num_heads, remaining_heads, ff_interm_features

    def forward(self, waveforms: Tensor, lengths: Optional[Tensor] = None) -> Tuple[Tensor, Optional[Tensor]]:
        """model.py:127-169."""
        if self.normalize_waveform:
            waveforms = self._normalize(waveforms, lengths)
        self._sample_gates()
        try:
            x, lengths = self.feature_extractor(waveforms, lengths)
            x = self.encoder(x, lengths)
        finally:
            self._drop_gates()
        if self.aux is not None:
            x = self.aux(x.float())
        return x, lengths


def wav2vec2_model(**configs) -> Wav2Vec2Model:
    """Wraps the original wav2vec2_model (model.py:172-178)."""
    m = wavlm_model(**configs) if "encoder_remaining_heads" in configs else wav2vec2_model_original(**configs)
    m.dph_config = dict(configs)       # (its FLOP / byte accounting in the training log: perfmodel)
    return m


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
