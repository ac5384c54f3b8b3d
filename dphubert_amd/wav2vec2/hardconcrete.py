"""HardConcrete L0 gate (drop-in for wav2vec2/hardconcrete.py of the reference).

Same constructor, parameter (``log_alpha``), ``forward()`` and ``l0_norm()``.
Training-mode sampling runs the HIP kernel ``dph_hc_sample_fwd`` (noise from a
counter-based generator, or an explicit ``u`` via ``set_noise`` for parity
runs); eval mode reproduces the deterministic top-k soft mask
(hardconcrete.py:101-114), which is host-side control logic (it needs
``.item()``) and only runs in eval / pruning.
"""

import math
from typing import Optional

import torch
import torch.nn as nn

from .. import ops


class HardConcrete(nn.Module):
    def __init__(self, n_in: int, init_mean: float = 0.5, init_std: float = 0.01, temperature: float = 2 / 3,
                 stretch: float = 0.1, eps: float = 1e-6) -> None:
        super().__init__()
        self.n_in = n_in
        self.limit_l = -stretch
        self.limit_r = 1.0 + stretch
        self.log_alpha = nn.Parameter(torch.zeros(n_in))
        self.beta = temperature
        self.init_mean = init_mean
        self.init_std = init_std
        self.bias = -self.beta * math.log(-self.limit_l / self.limit_r)
        self.eps = eps
        self.compiled_mask = None
        self._noise: Optional[torch.Tensor] = None
        self._bank_mask: Optional[torch.Tensor] = None   # this step's mask from the model's batched launch
        self.reset_parameters()

    def reset_parameters(self):
        self.compiled_mask = None
        mean = math.log(1 - self.init_mean) - math.log(self.init_mean)
        self.log_alpha.data.normal_(mean, self.init_std)

    def set_noise(self, u: Optional[torch.Tensor]):
        """Use an explicit uniform sample u (parity with a recorded reference run) for the next forwards."""
        self._noise = u

    def l0_norm(self) -> torch.Tensor:
        return (self.log_alpha + self.bias).sigmoid().sum()

    def forward(self) -> torch.Tensor:
        if self.training:
            self.compiled_mask = None
            if self._bank_mask is not None:      # sampled with every other gate of the model in one launch
                m, self._bank_mask = self._bank_mask, None
                return m
            if not self.log_alpha.is_cuda:
                raise RuntimeError("HardConcrete training-mode sampling runs on the GPU only (no CPU path)")
            u = self._noise
            if u is not None:
                u = u.to(self.log_alpha.device, torch.float32).contiguous()
            return ops.HardConcreteFn.apply(self.log_alpha, u)
        if self.compiled_mask is None:
            with torch.no_grad():
                expected_num_zeros = self.n_in - self.l0_norm().item()
                num_zeros = round(expected_num_zeros)
                soft_mask = torch.sigmoid(self.log_alpha / self.beta * 0.8)
                _, indices = torch.topk(soft_mask, k=num_zeros, largest=False)
                soft_mask[indices] = 0.0
                self.compiled_mask = soft_mask
        return self.compiled_mask

    def extra_repr(self) -> str:
        return str(self.n_in)

    def __repr__(self) -> str:
        return "{}({})".format(self.__class__.__name__, self.extra_repr())
