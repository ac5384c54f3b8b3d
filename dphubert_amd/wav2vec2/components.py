"""Model building blocks with pruning units (drop-in for wav2vec2/components.py).

Module names, parameter names / shapes / registration order, constructor
arguments and the ``prune()`` / ``get_num_params()`` surface follow the
reference, so checkpoints (``{'state_dict', 'config'}``) load unchanged.  The
modules here only *hold* parameters; every forward runs through the fused
autograd Functions of ``dphubert_amd.ops`` (HIP kernels, channels-last bf16
activations).  Layouts: feature tensors are (batch, frame, feature) bf16.
"""

from collections import defaultdict
from typing import Dict, List, Optional, Tuple

import torch
from torch import Tensor, nn
from torch.nn import Module

from .. import ops
from .hardconcrete import HardConcrete
from .pruning_utils import prune_conv1d_layer, prune_layer_norm, prune_linear_layer


# ---------------------------------------------------------------------------
# symbolic polynomial for the expected parameter count (get_num_params chain)
# ---------------------------------------------------------------------------
class Poly:
    """Sparse polynomial over HardConcrete l0 norms: {tuple(sorted var ids): coef}."""

    def __init__(self, terms=None):
        self.t: Dict[Tuple[int, ...], float] = dict(terms or {})

    @staticmethod
    def const(c) -> "Poly":
        return Poly({(): float(c)})

    @staticmethod
    def var(i: int) -> "Poly":
        return Poly({(i,): 1.0})

    def __add__(self, o):
        o = o if isinstance(o, Poly) else Poly.const(o)
        r = dict(self.t)
        for k, v in o.t.items():
            r[k] = r.get(k, 0.0) + v
        return Poly(r)

    __radd__ = __add__

    def __mul__(self, o):
        o = o if isinstance(o, Poly) else Poly.const(o)
        r: Dict[Tuple[int, ...], float] = {}
        for k1, v1 in self.t.items():
            for k2, v2 in o.t.items():
                k = tuple(sorted(k1 + k2))
                r[k] = r.get(k, 0.0) + v1 * v2
        return Poly(r)

    __rmul__ = __mul__


class _PolyCtx:
    """Assigns variable ids to HardConcrete modules in model order."""

    def __init__(self):
        self.mods: List[HardConcrete] = []

    def l0(self, hc: Optional[HardConcrete], default) -> Poly:
        if hc is None:
            return Poly.const(default)
        self.mods.append(hc)
        return Poly.var(len(self.mods) - 1)


# ---------------------------------------------------------------------------
class LayerNorm(nn.LayerNorm):
    """Layer norm over channels of a (batch, channel, frame) tensor (components.py:54-61)."""


class WeightNormConv1d(Module):
    """Parameter holder with the reference's weight_norm(dim=2) names: bias, weight_g, weight_v."""

    def __init__(self, channels: int, kernel_size: int, groups: int):
        super().__init__()
        self.in_channels = channels
        self.out_channels = channels
        self.kernel_size = (kernel_size,)
        self.groups = groups
        self.padding = (kernel_size // 2,)
        conv = nn.Conv1d(channels, channels, kernel_size, padding=kernel_size // 2, groups=groups)
        self.bias = nn.Parameter(conv.bias.detach().clone())
        w = conv.weight.detach()
        norm = w.pow(2).sum(dim=(0, 1), keepdim=True).sqrt()
        self.weight_g = nn.Parameter(norm.clone())
        self.weight_v = nn.Parameter(w.clone())

    def weight(self) -> Tensor:
        return self.weight_g * self.weight_v / self.weight_v.pow(2).sum(dim=(0, 1), keepdim=True).sqrt()


class ConvLayerBlock(Module):
    """Convolution unit of FeatureExtractor (components.py:64-134)."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int, bias: bool,
                 layer_norm: Optional[Module], prune_conv_channels: bool = False):
        super().__init__()
        self.kernel_size = kernel_size
        self.stride = stride
        self.layer_norm = layer_norm
        self.conv = nn.Conv1d(in_channels=in_channels, out_channels=out_channels, kernel_size=kernel_size,
                              stride=stride, bias=bias)
        if prune_conv_channels:
            self.hard_concrete = HardConcrete(n_in=out_channels, init_mean=0.01)
        else:
            self.hard_concrete = None

    def get_num_params_and_out_channels(self, in_channels):
        if self.hard_concrete is not None:
            out_channels = self.hard_concrete.l0_norm()
        else:
            out_channels = self.conv.out_channels
        num_params = in_channels * out_channels * self.kernel_size
        if self.conv.bias is not None:
            num_params += out_channels
        if self.layer_norm is not None:
            num_params += out_channels * 2
        return num_params, out_channels


class FeatureExtractor(Module):
    """Extract features from audio (components.py:137-235), fused into one HIP schedule."""

    def __init__(self, conv_layers: nn.ModuleList):
        super().__init__()
        self.conv_layers = conv_layers
        self.dummy_weight = nn.Parameter(torch.ones(conv_layers[-1].conv.out_channels, dtype=torch.float32),
                                         requires_grad=False)

    def _ln_mode(self) -> bool:
        """layer_norm-mode extractor (every conv layer carries a LayerNorm over channels)."""
        return all(isinstance(l.layer_norm, LayerNorm) for l in self.conv_layers)

    def _check_supported(self):
        if self._ln_mode():
            return
        l0 = self.conv_layers[0]
        if not isinstance(l0.layer_norm, nn.GroupNorm):
            raise NotImplementedError("mixed extractor normalisation is not on the HIP path")
        for layer in self.conv_layers:
            if layer.conv.bias is not None:
                raise NotImplementedError("conv bias (Large extractor) is not on the HIP path yet")
        for layer in list(self.conv_layers)[1:]:
            if layer.layer_norm is not None:
                raise NotImplementedError("per-layer conv LayerNorm is not on the HIP path yet")

    def forward(self, x: Tensor, length: Optional[Tensor]) -> Tuple[Tensor, Optional[Tensor]]:
        if x.ndim != 2:
            raise ValueError("Expected the input Tensor to be 2D (batch, time), " f"but received {list(x.shape)}")
        if not x.is_cuda:
            raise ValueError("FeatureExtractor runs on the MI355X HIP path only: pass a device tensor "
                             "(there is no CPU fallback)")
        self._check_supported()
        B, S = x.shape
        layers = [(l.conv.out_channels, l.kernel_size, l.stride) for l in self.conv_layers]
        masks = [l.hard_concrete() if l.hard_concrete is not None else None for l in self.conv_layers]
        l0 = self.conv_layers[0]
        need = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        cfg = ops.FrontendCfg(layers, B, S, need)
        flat = []
        if self._ln_mode():
            for l, m in zip(self.conv_layers, masks):
                flat += [l.conv.weight, l.conv.bias, l.layer_norm.weight, l.layer_norm.bias, m]
            y = ops.FrontendLNFn.apply(cfg, x.contiguous().float(), self.dummy_weight, *flat)
        else:
            for l, m in zip(self.conv_layers, masks):
                flat += [l.conv.weight, m]
            y = ops.FrontendFn.apply(cfg, x.contiguous().float(), self.dummy_weight, l0.layer_norm.weight,
                                     l0.layer_norm.bias, *flat)
        T = ops.conv_lengths(S, layers)[-1]
        C = layers[-1][0]
        Cp = ops.pad8(C)
        if Cp != C:
            # pruned (ragged) width: the HIP path keeps 8-padded rows; expose the reference's
            # (B, T, C) as a view and hand the padded storage to FeatureProjection
            yp = y
            y = yp.view(B, T, Cp)[:, :, :C]
            y._dph_padded = yp
        else:
            y = y.view(B, T, C)
        if length is not None:
            length = ops.conv_frame_lengths(length, layers)
        return y, length

    def get_num_params_and_final_out_channels(self):
        in_channels = 1
        num_params = 0
        for layer in self.conv_layers:
            layer_params, in_channels = layer.get_num_params_and_out_channels(in_channels)
            num_params += layer_params
        num_params += in_channels
        return num_params, in_channels

    def poly(self, ctx: _PolyCtx) -> Tuple[Poly, Poly]:
        in_c = Poly.const(1)
        total = Poly()
        for layer in self.conv_layers:
            oc = ctx.l0(layer.hard_concrete, layer.conv.out_channels)
            p = in_c * oc * layer.kernel_size
            if layer.conv.bias is not None:
                p = p + oc
            if layer.layer_norm is not None:
                p = p + oc * 2
            total = total + p
            in_c = oc
        return total + in_c, in_c

    def prune(self):
        """Eval-mode structural pruning (components.py:198-235)."""
        new_config = []
        index = None
        for idx, layer in enumerate(self.conv_layers):
            if layer.hard_concrete is not None:
                assert not layer.hard_concrete.training
                mask = layer.hard_concrete()
                index = mask.nonzero().squeeze(-1)
                assert len(index) > 0, f"Conv channels pruned to zero at index {idx}"
                new_config.append((len(index), layer.kernel_size, layer.stride))
                prune_conv1d_layer(layer.conv, index, "output")
                if layer.layer_norm is not None:
                    prune_layer_norm(layer.layer_norm, index)
                if idx == len(self.conv_layers) - 1:
                    self.dummy_weight.data *= mask
                    self.dummy_weight = nn.Parameter(self.dummy_weight.index_select(0, index).clone().detach(),
                                                     requires_grad=False)
                else:
                    self.conv_layers[idx + 1].conv.weight.data *= mask.unsqueeze(-1)
                    prune_conv1d_layer(self.conv_layers[idx + 1].conv, index, dim="input")
                layer.hard_concrete = None
            else:
                new_config.append((layer.conv.out_channels, layer.kernel_size, layer.stride))
                index = torch.arange(layer.conv.out_channels, dtype=torch.long)
        return new_config, index


class FeatureProjection(Module):
    """LayerNorm -> Linear -> Dropout (components.py:238-277)."""

    def __init__(self, in_features: int, out_features: int, dropout: float):
        super().__init__()
        self.layer_norm = nn.LayerNorm(in_features)
        self.projection = nn.Linear(in_features, out_features)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x, lengths: Optional[Tensor] = None):
        B, T, C = x.shape
        p = self.dropout.p if self.training else 0.0
        cfg = {"p": p, "lengths": lengths.to(x.device, torch.int64).contiguous() if lengths is not None else None,
               "T": T}
        xp = getattr(x, "_dph_padded", None)
        if xp is not None:
            cfg["C"] = C
        else:
            xp = x.reshape(B * T, C)
            if C % 4:
                raise NotImplementedError("FeatureProjection: ragged widths need the 8-padded frontend output")
        y = ops.FeatureProjectionFn.apply(xp, self.layer_norm.weight, self.layer_norm.bias,
                                          self.projection.weight, self.projection.bias, cfg)
        return y.view(B, T, -1)

    def get_num_params(self, in_features):
        return in_features * 2 + (in_features + 1) * self.projection.out_features


class ConvolutionalPositionalEmbedding(Module):
    """Grouped conv positional embedding with weight norm (components.py:280-333)."""

    def __init__(self, embed_dim: int, kernel_size: int, groups: int):
        super().__init__()
        self.embed_dim = embed_dim
        self.kernel_size = kernel_size
        self.groups = groups
        self.conv = WeightNormConv1d(embed_dim, kernel_size, groups)
        self.num_remove: int = 1 if kernel_size % 2 == 0 else 0


class SelfAttention(Module):
    """Multi-head self attention with head / layer HardConcrete masks (components.py:336-483)."""

    def __init__(self, embed_dim: int, num_heads: int, head_dim: int, dropout: float = 0.0,
                 prune_heads: bool = False, prune_layer: bool = False):
        super().__init__()
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.head_dim = head_dim
        self.dropout = torch.nn.Dropout(dropout)
        self.scaling = self.head_dim ** -0.5
        self.k_proj = nn.Linear(embed_dim, num_heads * head_dim, bias=True)
        self.v_proj = nn.Linear(embed_dim, num_heads * head_dim, bias=True)
        self.q_proj = nn.Linear(embed_dim, num_heads * head_dim, bias=True)
        self.out_proj = nn.Linear(num_heads * head_dim, embed_dim, bias=True)
        self.hard_concrete_for_heads = HardConcrete(n_in=num_heads, init_mean=0.01) if prune_heads else None
        self.hard_concrete_for_layer = HardConcrete(n_in=1, init_mean=0.01) if prune_layer else None

    def get_num_params(self):
        num_heads = self.hard_concrete_for_heads.l0_norm() if self.hard_concrete_for_heads is not None \
            else self.num_heads
        num_params = (self.embed_dim + 1) * num_heads * self.head_dim * 3 \
            + (num_heads * self.head_dim + 1) * self.embed_dim
        if self.hard_concrete_for_layer is not None:
            num_params *= self.hard_concrete_for_layer.l0_norm()
        return num_params

    def poly(self, ctx: _PolyCtx) -> Poly:
        nh = ctx.l0(self.hard_concrete_for_heads, self.num_heads)
        D, hd = self.embed_dim, self.head_dim
        p = nh * ((D + 1) * hd * 3) + (nh * hd + 1) * D
        if self.hard_concrete_for_layer is not None:
            p = p * ctx.l0(self.hard_concrete_for_layer, 1)
        return p

    def prune(self):
        new_config = {"use_attention": True, "num_heads": self.num_heads}
        if self.hard_concrete_for_layer is not None:
            assert not self.hard_concrete_for_layer.training
            layer_mask = self.hard_concrete_for_layer()
            self.out_proj.weight.data *= layer_mask
            self.out_proj.bias.data *= layer_mask
            if layer_mask == 0:
                new_config["use_attention"] = False
            self.hard_concrete_for_layer = None
        if self.hard_concrete_for_heads is not None:
            assert not self.hard_concrete_for_heads.training
            head_mask = self.hard_concrete_for_heads()
            new_config["num_heads"] = len(head_mask.nonzero())
            if new_config["num_heads"] == 0:
                new_config["use_attention"] = False
            else:
                full_mask = head_mask.repeat_interleave(self.head_dim)
                full_index = full_mask.nonzero().squeeze(-1)
                prune_linear_layer(self.k_proj, full_index, "output")
                prune_linear_layer(self.v_proj, full_index, "output")
                prune_linear_layer(self.q_proj, full_index, "output")
                self.out_proj.weight.data *= full_mask
                prune_linear_layer(self.out_proj, full_index, "input")
            self.hard_concrete_for_heads = None
        return new_config


class WavLMSelfAttention(SelfAttention):
    """WavLM attention (components.py:486-693): SelfAttention over ``remaining_heads`` of ``total_num_heads`` plus
    the gated relative-position bias.  Layer 0 owns ``rel_attn_embed`` (num_buckets x total heads); its bucketed
    table (``ops.RelPosTableFn``, one value per diagonal) is the ``position_bias`` handed to every later layer,
    and each layer gates it per query (``gru_rel_pos_linear`` / ``gru_rel_pos_const``) inside the attention
    kernels -- no (B*H, T, T) tensor is built.  Parameter names and registration order follow the reference."""

    def __init__(self, embed_dim: int, total_num_heads: int, remaining_heads: Optional[List[int]] = None,
                 dropout: float = 0.0, bias: bool = True, has_relative_attention_bias: bool = False,
                 num_buckets: int = 32, max_distance: int = 128, gru_rel_pos: bool = True,
                 prune_heads: bool = False, prune_layer: bool = False):
        self.total_num_heads = total_num_heads
        self.remaining_heads = list(range(total_num_heads)) if remaining_heads is None else list(remaining_heads)
        head_dim = embed_dim // total_num_heads
        super().__init__(embed_dim, len(self.remaining_heads), head_dim, dropout, prune_heads, prune_layer)
        if not bias:
            raise NotImplementedError("WavLMSelfAttention(bias=False): the reference builder always uses bias")
        if not gru_rel_pos:
            raise NotImplementedError("WavLMSelfAttention(gru_rel_pos=False): the reference builder always gates")
        self.has_relative_attention_bias = has_relative_attention_bias
        self.num_buckets = num_buckets
        self.max_distance = max_distance
        self.rel_attn_embed = nn.Embedding(num_buckets, total_num_heads) if has_relative_attention_bias else None
        self.gru_rel_pos = gru_rel_pos
        self.gru_rel_pos_linear = nn.Linear(head_dim, 8)
        self.gru_rel_pos_const = nn.Parameter(torch.ones(1, total_num_heads, 1, 1))
        self.has_position_bias = True
        self._heads_dev = None

    def heads_tensor(self, dev) -> Optional[Tensor]:
        """int64 device tensor of the remaining heads' indices (None when every head remains)."""
        if self.remaining_heads == list(range(self.total_num_heads)):
            return None
        if self._heads_dev is None or self._heads_dev.device != dev:
            self._heads_dev = torch.tensor(self.remaining_heads, dtype=torch.int64, device=dev)
        return self._heads_dev

    def prune(self):
        """components.py:661-693 (``remaining_heads`` = nonzero head-mask indices, as the reference)."""
        new_config = {"use_attention": True, "remaining_heads": self.remaining_heads}
        if self.hard_concrete_for_layer is not None:
            assert not self.hard_concrete_for_layer.training
            layer_mask = self.hard_concrete_for_layer()
            self.out_proj.weight.data *= layer_mask
            self.out_proj.bias.data *= layer_mask
            if layer_mask == 0:
                new_config["use_attention"] = False
            self.hard_concrete_for_layer = None
        if self.hard_concrete_for_heads is not None:
            assert not self.hard_concrete_for_heads.training
            head_mask = self.hard_concrete_for_heads()
            new_config["remaining_heads"] = head_mask.nonzero().squeeze(-1).tolist()
            if len(new_config["remaining_heads"]) == 0:
                new_config["use_attention"] = False
            else:
                full_mask = head_mask.repeat_interleave(self.head_dim)
                full_index = full_mask.nonzero().squeeze(-1)
                prune_linear_layer(self.k_proj, full_index, "output")
                prune_linear_layer(self.v_proj, full_index, "output")
                prune_linear_layer(self.q_proj, full_index, "output")
                self.out_proj.weight.data *= full_mask
                prune_linear_layer(self.out_proj, full_index, "input")
            self.hard_concrete_for_heads = None
        return new_config


class FeedForward(Module):
    """Linear -> GELU -> dropout -> x interm mask -> Linear -> dropout -> x layer mask (components.py:696-791)."""

    def __init__(self, io_features: int, intermediate_features: int, intermediate_dropout: float,
                 output_dropout: float, prune_intermediate: bool = False, prune_layer: bool = False):
        super().__init__()
        self.intermediate_dense = nn.Linear(io_features, intermediate_features)
        self.intermediate_dropout = nn.Dropout(intermediate_dropout)
        self.output_dense = nn.Linear(intermediate_features, io_features)
        self.output_dropout = nn.Dropout(output_dropout)
        self.hard_concrete_for_intermediate = HardConcrete(n_in=intermediate_features, init_mean=0.5) \
            if prune_intermediate else None
        self.hard_concrete_for_layer = HardConcrete(n_in=1, init_mean=0.01) if prune_layer else None

    def get_num_params(self):
        io_features = self.intermediate_dense.in_features
        f = self.hard_concrete_for_intermediate.l0_norm() if self.hard_concrete_for_intermediate is not None \
            else self.intermediate_dense.out_features
        num_params = (io_features + 1) * f + (f + 1) * io_features
        if self.hard_concrete_for_layer is not None:
            num_params *= self.hard_concrete_for_layer.l0_norm()
        return num_params

    def poly(self, ctx: _PolyCtx) -> Poly:
        D = self.intermediate_dense.in_features
        f = ctx.l0(self.hard_concrete_for_intermediate, self.intermediate_dense.out_features)
        p = f * (D + 1) + (f + 1) * D
        if self.hard_concrete_for_layer is not None:
            p = p * ctx.l0(self.hard_concrete_for_layer, 1)
        return p

    def prune(self):
        new_config = {"use_feed_forward": True, "ff_interm_features": self.intermediate_dense.out_features}
        if self.hard_concrete_for_layer is not None:
            assert not self.hard_concrete_for_layer.training
            layer_mask = self.hard_concrete_for_layer()
            self.output_dense.weight.data *= layer_mask
            self.output_dense.bias.data *= layer_mask
            if layer_mask == 0:
                new_config["use_feed_forward"] = False
            self.hard_concrete_for_layer = None
        if self.hard_concrete_for_intermediate is not None:
            assert not self.hard_concrete_for_intermediate.training
            interm_mask = self.hard_concrete_for_intermediate()
            interm_index = interm_mask.nonzero().squeeze(-1)
            new_config["ff_interm_features"] = len(interm_index)
            if new_config["ff_interm_features"] == 0:
                new_config["use_feed_forward"] = False
            else:
                prune_linear_layer(self.intermediate_dense, interm_index, "output")
                self.output_dense.weight.data *= interm_mask
                prune_linear_layer(self.output_dense, interm_index, "input")
            self.hard_concrete_for_intermediate = None
        return new_config


class EncoderLayer(Module):
    """Attention + FFN block, post-norm (Base) or pre-norm (Large) (components.py:794-865)."""

    def __init__(self, attention: Optional[Module], dropout: float, layer_norm_first: bool,
                 feed_forward: Optional[Module], embed_dim: int):
        super().__init__()
        self.attention = attention
        self.dropout = nn.Dropout(dropout)
        self.layer_norm = nn.LayerNorm(embed_dim)
        self.layer_norm_first = layer_norm_first
        self.feed_forward = feed_forward
        self.final_layer_norm = nn.LayerNorm(embed_dim)
        self.embed_dim = embed_dim

    def forward(self, x: Tensor, attention_mask=None, position_bias: Optional[Tensor] = None,
                key_padding_mask: Optional[Tensor] = None, key_len: Optional[Tensor] = None):
        B, T, D = x.shape
        att, ff = self.attention, self.feed_forward
        tr = self.training
        if att is not None and (x.ndim != 3 or D != att.embed_dim):
            raise ValueError(f"The expected input shape is (batch, sequence, embed_dim=={att.embed_dim}). "
                             f"Found {x.shape}.")
        hm = att.hard_concrete_for_heads() if (att is not None and att.hard_concrete_for_heads is not None) else None
        lma = att.hard_concrete_for_layer() if (att is not None and att.hard_concrete_for_layer is not None) else None
        im = ff.hard_concrete_for_intermediate() if (ff is not None and ff.hard_concrete_for_intermediate is not None) \
            else None
        lmf = ff.hard_concrete_for_layer() if (ff is not None and ff.hard_concrete_for_layer is not None) else None
        need = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        cfg = {
            "need_grad": need, "B": B, "T": T,
            "H": att.num_heads if att is not None else 0,
            "head_dim": att.head_dim if att is not None else 64,
            "p_attn": att.dropout.p if (tr and att is not None) else 0.0,
            "p_drop": self.dropout.p if tr else 0.0,
            "p_interm": ff.intermediate_dropout.p if (tr and ff is not None) else 0.0,
            "lengths": key_len,
            "pre_norm": bool(self.layer_norm_first),
            # FFN GEMMs over the active units only (ops._ffn_forward): the trainer sets this per gate from its
            # expected zero fraction (Trainer.refresh_ffn_compaction)
            "ffn_compact": bool(getattr(ff.hard_concrete_for_intermediate, "dph_compact", False))
            if (ff is not None and ff.hard_concrete_for_intermediate is not None) else False,
        }
        if ff is not None and tr and ff.output_dropout.p != self.dropout.p:
            raise NotImplementedError("FFN output dropout != layer dropout")
        rel_tab = gw = gb = gc = heads = None
        if isinstance(att, WavLMSelfAttention):
            # components.py:629-631: only the layer owning the embedding builds the bias, and only when none was
            # handed in (a dropped layer 0 leaves every later layer without one, as in the reference)
            if att.rel_attn_embed is not None and position_bias is None:
                position_bias = ops.RelPosTableFn.apply(att.rel_attn_embed.weight, T, att.num_buckets,
                                                        att.max_distance)
            if position_bias is not None:
                heads = att.heads_tensor(x.device)
                rel_tab = position_bias if heads is None else position_bias.index_select(0, heads)
                gw, gb, gc = att.gru_rel_pos_linear.weight, att.gru_rel_pos_linear.bias, att.gru_rel_pos_const
                cfg["wavlm"] = True
        a = att
        out = ops.EncoderLayerFn.apply(
            cfg, x.reshape(B * T, D),
            a.q_proj.weight if a else None, a.k_proj.weight if a else None, a.v_proj.weight if a else None,
            a.q_proj.bias if a else None, a.k_proj.bias if a else None, a.v_proj.bias if a else None,
            a.out_proj.weight if a else None, a.out_proj.bias if a else None,
            self.layer_norm.weight, self.layer_norm.bias,
            ff.intermediate_dense.weight if ff else None, ff.intermediate_dense.bias if ff else None,
            ff.output_dense.weight if ff else None, ff.output_dense.bias if ff else None,
            self.final_layer_norm.weight, self.final_layer_norm.bias, hm, lma, im, lmf, rel_tab, gw, gb, gc, heads)
        return out.view(B, T, D), position_bias

    def get_num_params(self):
        num_params = self.embed_dim * 2 * 2
        if self.attention is not None:
            num_params += self.attention.get_num_params()
        if self.feed_forward is not None:
            num_params += self.feed_forward.get_num_params()
        return num_params

    def poly(self, ctx: _PolyCtx) -> Poly:
        p = Poly.const(self.embed_dim * 2 * 2)
        if self.attention is not None:
            p = p + self.attention.poly(ctx)
        if self.feed_forward is not None:
            p = p + self.feed_forward.poly(ctx)
        return p


class Transformer(Module):
    def __init__(self, pos_conv_embed: Module, dropout: float, layers: Module, layer_norm_first: bool,
                 layer_drop: float):
        super().__init__()
        self.pos_conv_embed = pos_conv_embed
        self.layer_norm = nn.LayerNorm(pos_conv_embed.embed_dim)
        self.layer_norm_first = layer_norm_first
        self.layer_drop = layer_drop
        self.dropout = nn.Dropout(dropout)
        self.layers = layers

    def _preprocess(self, x: Tensor):
        """x + pos_conv(x) -> [LayerNorm] -> dropout (components.py:885-892): the LN runs for post-norm
        (Base) encoders only -- the flag is inverted at construction (components.py:1283)."""
        B, T, D = x.shape
        pc = self.pos_conv_embed
        need = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        cfg = {"B": B, "T": T, "G": pc.groups, "p": self.dropout.p if self.training else 0.0, "need_grad": need,
               "ln": bool(self.layer_norm_first)}
        h = ops.PosConvFn.apply(x.reshape(B * T, D), pc.conv.weight_g, pc.conv.weight_v, pc.conv.bias,
                                self.layer_norm.weight, self.layer_norm.bias, cfg)
        return h.view(B, T, D)

    def forward(self, x: Tensor, attention_mask=None, position_bias=None, key_len=None) -> Tensor:
        import random
        x = ops.mark_encoder_input(self._preprocess(x))
        for layer in self.layers:
            if not (self.training and random.random() <= self.layer_drop):
                x, position_bias = layer(x, attention_mask, position_bias=position_bias, key_len=key_len)
        if not self.layer_norm_first:
            B, T, D = x.shape
            x = ops.LayerNormFn.apply(x.reshape(B * T, D), self.layer_norm.weight, self.layer_norm.bias).view(B, T, D)
        return x

    def get_intermediate_outputs(self, x: Tensor, attention_mask=None, num_layers: Optional[int] = None,
                                 position_bias=None, key_len=None) -> List[Tensor]:
        if num_layers is not None:
            if not 0 < num_layers <= len(self.layers):
                raise ValueError(f"`num_layers` must be between [1, {len(self.layers)}]")
        ret: List[Tensor] = []
        x = ops.mark_encoder_input(self._preprocess(x))
        for layer in self.layers:
            x, position_bias = layer(x, attention_mask, position_bias=position_bias, key_len=key_len)
            ret.append(x)
            if num_layers is not None and len(ret) >= num_layers:
                return ret
        return ret

    def get_num_params(self):
        num_params = sum(p.numel() for p in self.pos_conv_embed.parameters()) + self.pos_conv_embed.embed_dim * 2
        for layer in self.layers:
            num_params += layer.get_num_params()
        return num_params

    def poly(self, ctx: _PolyCtx) -> Poly:
        p = Poly.const(sum(q.numel() for q in self.pos_conv_embed.parameters()) + self.pos_conv_embed.embed_dim * 2)
        for layer in self.layers:
            p = p + layer.poly(ctx)
        return p

    def prune(self):
        new_config = defaultdict(list)
        for layer in self.layers:
            attention_config = layer.attention.prune()
            new_config["use_attention"].append(attention_config["use_attention"])
            if "remaining_heads" in attention_config:
                new_config["remaining_heads"].append(attention_config["remaining_heads"])
            else:
                new_config["num_heads"].append(attention_config["num_heads"])
            if not attention_config["use_attention"]:
                layer.attention = None
            ff_config = layer.feed_forward.prune()
            new_config["use_feed_forward"].append(ff_config["use_feed_forward"])
            new_config["ff_interm_features"].append(ff_config["ff_interm_features"])
            if not ff_config["use_feed_forward"]:
                layer.feed_forward = None
        return new_config


class Encoder(Module):
    def __init__(self, feature_projection: Module, transformer: Module):
        super().__init__()
        self.feature_projection = feature_projection
        self.transformer = transformer

    def _preprocess(self, features: Tensor, lengths: Optional[Tensor] = None):
        """components.py:968-984: projection, zero padded frames; the additive -1e4 key mask is applied
        inside the attention kernel from the key lengths instead of a materialised (B,1,T,T) tensor."""
        x = self.feature_projection(features, lengths)
        key_len = None
        if lengths is not None:
            key_len = lengths.to(x.device, torch.int64).contiguous()
        return x, key_len

    def forward(self, features: Tensor, lengths: Optional[Tensor] = None) -> Tensor:
        x, key_len = self._preprocess(features, lengths)
        return self.transformer(x, key_len=key_len)

    def extract_features(self, features: Tensor, lengths: Optional[Tensor] = None,
                         num_layers: Optional[int] = None) -> List[Tensor]:
        x, key_len = self._preprocess(features, lengths)
        interm = self.transformer.get_intermediate_outputs(x, num_layers=num_layers, key_len=key_len)
        return [x] + interm

    def get_num_params(self, in_features):
        return self.feature_projection.get_num_params(in_features) + self.transformer.get_num_params()

    def poly(self, ctx: _PolyCtx, in_features: Poly) -> Poly:
        D = self.feature_projection.projection.out_features
        return in_features * 2 + (in_features + 1) * D + self.transformer.poly(ctx)

    def prune(self, conv_out_index):
        prune_layer_norm(self.feature_projection.layer_norm, conv_out_index)
        prune_linear_layer(self.feature_projection.projection, conv_out_index, "input")
        return self.transformer.prune()


# ---------------------------------------------------------------------------
def _get_feature_extractor(norm_mode: str, shapes: List[Tuple[int, int, int]], bias: bool,
                           prune_conv_channels: bool = False) -> FeatureExtractor:
    if norm_mode not in ["group_norm", "layer_norm"]:
        raise ValueError("Invalid norm mode")
    blocks = []
    in_channels = 1
    for i, (out_channels, kernel_size, stride) in enumerate(shapes):
        normalization = None
        if norm_mode == "group_norm" and i == 0:
            normalization = nn.GroupNorm(num_groups=out_channels, num_channels=out_channels, affine=True)
        elif norm_mode == "layer_norm":
            normalization = LayerNorm(normalized_shape=out_channels, elementwise_affine=True)
        blocks.append(ConvLayerBlock(in_channels=in_channels, out_channels=out_channels, kernel_size=kernel_size,
                                     stride=stride, bias=bias, layer_norm=normalization,
                                     prune_conv_channels=prune_conv_channels))
        in_channels = out_channels
    return FeatureExtractor(nn.ModuleList(blocks))


def _get_wavlm_encoder(in_features: int, embed_dim: int, dropout_input: float, pos_conv_kernel: int,
                       pos_conv_groups: int, num_layers: int, use_attention: List[bool], use_feed_forward: List[bool],
                       total_num_heads: List[int], remaining_heads: List[List[int]], num_buckets: int,
                       max_distance: int, attention_dropout: float, ff_interm_features: List[int],
                       ff_interm_dropout: float, dropout: float, layer_norm_first: bool, layer_drop: float,
                       prune_attention_heads: bool = False, prune_attention_layer: bool = False,
                       prune_feed_forward_intermediate: bool = False,
                       prune_feed_forward_layer: bool = False) -> Encoder:
    """components.py:1289-1386: the wav2vec2 encoder with WavLMSelfAttention (relative-position embedding in
    layer 0 only)."""
    feature_projection = FeatureProjection(in_features, embed_dim, dropout_input)
    pos_conv = ConvolutionalPositionalEmbedding(embed_dim, pos_conv_kernel, pos_conv_groups)
    encoder_layers = nn.ModuleList()
    for i in range(num_layers):
        attention = WavLMSelfAttention(embed_dim=embed_dim, total_num_heads=total_num_heads[i],
                                       remaining_heads=remaining_heads[i], dropout=attention_dropout,
                                       has_relative_attention_bias=(i == 0), num_buckets=num_buckets,
                                       max_distance=max_distance, prune_heads=prune_attention_heads,
                                       prune_layer=prune_attention_layer) if use_attention[i] else None
        feed_forward = FeedForward(io_features=embed_dim, intermediate_features=ff_interm_features[i],
                                   intermediate_dropout=ff_interm_dropout, output_dropout=dropout,
                                   prune_intermediate=prune_feed_forward_intermediate,
                                   prune_layer=prune_feed_forward_layer) if use_feed_forward[i] else None
        encoder_layers.append(EncoderLayer(attention=attention, dropout=dropout, layer_norm_first=layer_norm_first,
                                           feed_forward=feed_forward, embed_dim=embed_dim))
    transformer = Transformer(pos_conv_embed=pos_conv, dropout=dropout, layers=encoder_layers,
                              layer_norm_first=not layer_norm_first, layer_drop=layer_drop)
    return Encoder(feature_projection, transformer)


def _get_encoder(in_features: int, embed_dim: int, dropout_input: float, pos_conv_kernel: int,
                 pos_conv_groups: int, num_layers: int, use_attention: List[bool], use_feed_forward: List[bool],
                 num_heads: List[int], head_dim: int, attention_dropout: float, ff_interm_features: List[int],
                 ff_interm_dropout: float, dropout: float, layer_norm_first: bool, layer_drop: float,
                 prune_attention_heads: bool = False, prune_attention_layer: bool = False,
                 prune_feed_forward_intermediate: bool = False, prune_feed_forward_layer: bool = False) -> Encoder:
    feature_projection = FeatureProjection(in_features, embed_dim, dropout_input)
    pos_conv = ConvolutionalPositionalEmbedding(embed_dim, pos_conv_kernel, pos_conv_groups)
    encoder_layers = nn.ModuleList()
    for idx in range(num_layers):
        attention = SelfAttention(embed_dim=embed_dim, num_heads=num_heads[idx], head_dim=head_dim,
                                  dropout=attention_dropout, prune_heads=prune_attention_heads,
                                  prune_layer=prune_attention_layer) if use_attention[idx] else None
        feed_forward = FeedForward(io_features=embed_dim, intermediate_features=ff_interm_features[idx],
                                   intermediate_dropout=ff_interm_dropout, output_dropout=dropout,
                                   prune_intermediate=prune_feed_forward_intermediate,
                                   prune_layer=prune_feed_forward_layer) if use_feed_forward[idx] else None
        encoder_layers.append(EncoderLayer(attention=attention, dropout=dropout, layer_norm_first=layer_norm_first,
                                           feed_forward=feed_forward, embed_dim=embed_dim))
    # the reference inverts the flag here (components.py:1283): Base applies the LN in _preprocess
    transformer = Transformer(pos_conv_embed=pos_conv, dropout=dropout, layers=encoder_layers,
                              layer_norm_first=not layer_norm_first, layer_drop=layer_drop)
    return Encoder(feature_projection, transformer)
