"""Training-loop glue: builds the distill.py objects and runs one optimizer step.

Mirrors what PyTorch-Lightning did around ``DistillModule`` in the reference
(distill.py:29-144, final_distill.py:24-128): teacher (frozen) + student
(+ HardConcrete units) from ``{'state_dict','config'}`` checkpoints or from
seeded weights, identity-initialised per-group distill projections
(distill.py:24-26, 86-99), ``configure_optimizers`` (AdamW groups +
LinearDecayLR), gradient clipping, and the data-parallel all-reduce
(``dphubert_amd.ddp.GradReducer`` over RCCL).
"""

import copy
from typing import List, Optional

import torch
import torch.nn as nn

from . import ops
from .ddp import GradReducer
from .lightning import DistillLoss, DistillModule
from .synthetic import seeded_state_dict
from .wav2vec2.model import wav2vec2_model


def units_flags(pruning_units: str) -> dict:
    units = pruning_units.split(",") if pruning_units else []
    return dict(extractor_prune_conv_channels="conv" in units, encoder_prune_attention_heads="head" in units,
                encoder_prune_attention_layer="attlayer" in units,
                encoder_prune_feed_forward_intermediate="interm" in units,
                encoder_prune_feed_forward_layer="ffnlayer" in units)


def build_projections(distill_layers: str, d_student: int, d_teacher: int, identity_init: bool = True):
    """distill.py:86-99: one Linear per period-separated group, shared inside the group."""
    groups = [[int(l) for l in g.split(",")] for g in distill_layers.split(".")]
    layers, projs = [], nn.ModuleList()
    for g in groups:
        lin = nn.Linear(d_student, d_teacher)
        if identity_init:
            with torch.no_grad():
                lin.weight.copy_(torch.eye(len(lin.weight)))
                lin.bias.fill_(0)
        for l in g:
            layers.append(l)
            projs.append(lin)
    return layers, projs


def seeded_model(config: dict, seed: int = 0):
    m = wav2vec2_model(**copy.deepcopy(config))
    sd = seeded_state_dict([(k, tuple(v.shape)) for k, v in m.state_dict().items()], seed)
    m.load_state_dict(sd)
    return m


def build_distill_module(teacher_config: dict, student_config: Optional[dict] = None, *, pruning_units: str =
                         "conv,head,interm", distill_layers: str = "0.4,8,12", use_reg: bool = True,
                         teacher_state: Optional[dict] = None, student_state: Optional[dict] = None,
                         seed: int = 0, l2_weight: float = 0.0, l1_weight: float = 1.0, cos_weight: float = 1.0,
                         cos_type: str = "raw", learning_rate: float = 2e-4, weight_decay: float = 0.0,
                         warmup_updates: int = 15000, max_updates: int = 50000, reg_learning_rate: float = 0.02,
                         target_sparsity: float = 0.75, sparsity_warmup_updates: int = 5000,
                         proj_state: Optional[dict] = None) -> DistillModule:
    teacher = wav2vec2_model(**copy.deepcopy(teacher_config))
    if teacher_state is not None:
        teacher.load_state_dict(teacher_state, strict=False)
    else:
        teacher = seeded_model(teacher_config, seed)
    for p in teacher.parameters():
        p.requires_grad = False
    teacher.eval()
    scfg = copy.deepcopy(student_config if student_config is not None else teacher_config)
    if use_reg:
        scfg.update(units_flags(pruning_units))
    student = wav2vec2_model(**scfg)
    if student_state is not None:
        student.load_state_dict(student_state, strict=False)
    else:
        # student initialised from the teacher (run.sh:20), HardConcrete logits per reference init
        seeded = seeded_model(scfg, seed)
        student.load_state_dict(seeded.state_dict())
    layers, projs = build_projections(distill_layers, student.encoder.feature_projection.projection.out_features,
                                      teacher.encoder.feature_projection.projection.out_features,
                                      identity_init=proj_state is None)
    if proj_state is not None:
        projs.load_state_dict(proj_state)
    return DistillModule(teacher_model=teacher, student_model=student, distill_mode="layer2layer",
                         distill_layers=layers, distill_linear_projs=projs,
                         distill_loss=DistillLoss(l2_weight, l1_weight, cos_weight, cos_type),
                         learning_rate=learning_rate, weight_decay=weight_decay, warmup_updates=warmup_updates,
                         max_updates=max_updates, use_reg=use_reg,
                         reg_learning_rate=reg_learning_rate if use_reg else None,
                         target_sparsity=target_sparsity if use_reg else None,
                         sparsity_warmup_updates=sparsity_warmup_updates if use_reg else None)


def fused_grad_groups(model) -> List[tuple]:
    """Parameters whose gradients one fused kernel produces together (q/k/v weight and bias
    gradients come out of a single [3*Dh, D] weight-gradient GEMM / column sum)."""
    groups = []
    for layer in model.encoder.transformer.layers:
        a = layer.attention
        if a is not None:
            groups.append((a.q_proj.weight, a.k_proj.weight, a.v_proj.weight))
            groups.append((a.q_proj.bias, a.k_proj.bias, a.v_proj.bias))
    return groups


class Trainer:
    """One process per GPU; call ``step(batch)`` per optimizer update (accum_grad=1)."""

    def __init__(self, module: DistillModule, clip_norm: float = 10.0, bucket_mb: float = 64.0,
                 accum_grad: int = 1):
        self.module = module
        opt = module.configure_optimizers(clip_norm=clip_norm)
        self.optimizer = opt["optimizer"]
        self.scheduler = opt["lr_scheduler"]["scheduler"]
        params = [p for g in self.optimizer.param_groups for p in g["params"]]
        self.reducer = GradReducer(params, bucket_mb=bucket_mb, groups=fused_grad_groups(module.student_model))
        self.accum_grad = accum_grad
        self._micro = 0

    def step(self, batch):
        m = self.module
        m.train()
        self.reducer.prepare(zero=self._micro == 0, sync=self._micro + 1 == self.accum_grad)
        loss = m.training_step(batch, 0)
        (loss / self.accum_grad if self.accum_grad > 1 else loss).backward()
        self._micro += 1
        if self._micro < self.accum_grad:
            return loss
        self._micro = 0
        self.reducer.finish()
        self.optimizer.step()
        self.scheduler.step()
        for g in self.optimizer.param_groups:
            for p in g["params"]:
                p.grad = None
        m.global_step += 1
        return loss
