"""In-place structural pruning helpers (mirror of wav2vec2/pruning_utils.py:9-51).

Offline, one-shot host logic (index_select of kept rows / columns); not on the
training hot path.
"""

from typing import Union

import torch
import torch.nn as nn


def _select(t: torch.Tensor, dim: int, index: torch.LongTensor) -> nn.Parameter:
    return nn.Parameter(t.index_select(dim, index.to(t.device)).clone().detach())


def prune_linear_layer(layer: nn.Linear, index: torch.LongTensor, dim: str):
    """Keep ``index`` along the output (dim 0) or input (dim 1) features of a Linear."""
    if dim not in ("input", "output"):
        raise ValueError
    d = 1 if dim == "input" else 0
    if d == 1:
        layer.in_features = len(index)
    else:
        layer.out_features = len(index)
    layer.weight = _select(layer.weight, d, index)
    if layer.bias is not None and d == 0:
        layer.bias = _select(layer.bias, 0, index)


def prune_conv1d_layer(layer: nn.Conv1d, index: torch.LongTensor, dim: str):
    """Keep ``index`` along the output (dim 0) or input (dim 1) channels of a Conv1d."""
    if dim not in ("input", "output"):
        raise ValueError
    d = 1 if dim == "input" else 0
    if d == 1:
        layer.in_channels = len(index)
    else:
        layer.out_channels = len(index)
    layer.weight = _select(layer.weight, d, index)
    if layer.bias is not None and d == 0:
        layer.bias = _select(layer.bias, 0, index)


def prune_layer_norm(layernorm: Union[nn.LayerNorm, nn.GroupNorm], index: torch.LongTensor):
    """Keep ``index`` channels of a LayerNorm / GroupNorm (one group per channel)."""
    layernorm.weight = _select(layernorm.weight, 0, index)
    layernorm.bias = _select(layernorm.bias, 0, index)
    if isinstance(layernorm, nn.LayerNorm):
        layernorm.normalized_shape = (len(index),)
    elif isinstance(layernorm, nn.GroupNorm):
        layernorm.num_groups = len(index)
        layernorm.num_channels = len(index)
