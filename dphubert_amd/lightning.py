"""Distillation + pruning training module (drop-in for lightning.py of the reference).

``DistillModule`` keeps the reference constructor (lightning.py:142-198), the
``_step`` semantics (lightning.py:245-296: teacher forward under no_grad,
student forward, per-layer projection, DistillLoss, Lagrangian regulariser
on the expected sparsity) and ``configure_optimizers`` (3 AdamW groups +
linear warmup/decay).  It is a plain ``nn.Module`` with the few
LightningModule hooks the reference uses (``global_step``, ``log_dict``,
``training_step``); pytorch_lightning is not installed here, and the
multi-GPU loop lives in ``dphubert_amd.trainer`` (RCCL over xGMI).

On the hot path the projection + loss run fused on the GPU
(``ops.DistillProjLossFn``: projection GEMMs write straight into the loss
input, teacher layers are read in place, no ``torch.stack`` copies).
"""

import contextlib
import math
import pathlib
from typing import List, Optional, Union

import torch
import torch.nn as nn

from . import ops
from .optim import FusedAdamW, LinearDecayLRScheduler
from .wav2vec2.model import Wav2Vec2Model

__all__ = ["DistillLoss", "DistillModule", "LinearDecayLRScheduler"]

_TEACHER_AFTER = __import__("os").environ.get("DPH_TEACHER_ORDER", "before") == "after"


class DistillLoss(nn.Module):
    """lightning.py:91-139: ``loss = l2*MSE + l1*L1 + cos*(-mean cos)`` (or the ``log_sig`` variant)."""

    def __init__(self, l2_weight, l1_weight, cos_weight, cos_type):
        super().__init__()
        self.l2_weight = l2_weight
        self.l1_weight = l1_weight
        self.cos_weight = cos_weight
        self.cos_type = cos_type
        assert cos_type in ["raw", "log_sig"], cos_type

    def __repr__(self) -> str:
        return "{}(l2={}, l1={}, {}_cos={})".format(self.__class__.__name__, self.l2_weight, self.l1_weight,
                                                    self.cos_type, self.cos_weight)

    def cfg(self):
        return {"l2": float(self.l2_weight), "l1": float(self.l1_weight), "cos": float(self.cos_weight),
                "cos_type": self.cos_type}

    def forward(self, input: torch.Tensor, target: torch.Tensor):
        """input/target: (batch, layer, time, feature).  Returns (loss, (mse, l1, cos))."""
        if input.ndim != 4 or input.shape != target.shape:
            raise ValueError("DistillLoss expects matching (batch, layer, time, feature) tensors")
        B, L, T, D = input.shape
        s = input.float().permute(1, 0, 2, 3).contiguous()          # layer-major rows (loss is row-order free)
        t_layers = [target[:, l].to(torch.bfloat16).contiguous() for l in range(L)]
        loss, mse, l1, cos = _LossOnlyFn.apply(self.cfg(), B, T, s, *t_layers)
        return loss, (mse, l1, cos)


class _LossOnlyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, B, T, s, *t_layers):
        from ._lib import C as _C, call, ptr
        L, D = s.shape[0], s.shape[-1]
        dev = s.device
        rowstats = torch.empty(L * B * T * 3, dtype=torch.float32, device=dev)
        partial = torch.empty(ops.LOSS_PARTIAL_FLOATS, dtype=torch.float32, device=dev)
        out = torch.empty(4, dtype=torch.float32, device=dev)
        tptrs = (_C.c_void_p * L)(*[t.data_ptr() for t in t_layers])
        call("dph_distill_loss_fwd", ptr(s), tptrs, B, L, T, D, cfg["l2"], cfg["l1"], cfg["cos"],
             int(cfg["cos_type"] == "log_sig"), ptr(rowstats), ptr(partial), ptr(out), ops._s())
        ctx.cfg = (cfg, B, T, L, D)
        ctx.save_for_backward(s, rowstats, *t_layers)
        return out[0], out[1], out[2], out[3]

    @staticmethod
    def backward(ctx, dloss, *_):
        from ._lib import C as _C, call, ptr
        cfg, B, T, L, D = ctx.cfg
        s, rowstats, *t_layers = ctx.saved_tensors
        ds = torch.empty(s.shape, dtype=torch.bfloat16, device=s.device)
        tptrs = (_C.c_void_p * L)(*[t.data_ptr() for t in t_layers])
        call("dph_distill_loss_bwd", ptr(s), tptrs, ptr(rowstats), ptr(dloss.contiguous()), B, L, T, D, cfg["l2"],
             cfg["l1"], cfg["cos"], int(cfg["cos_type"] == "log_sig"), ptr(ds), ops._s())
        return (None, None, None, ds.float()) + (None,) * len(t_layers)


class DistillModule(nn.Module):
    """lightning.py:142-342 (training-step math; data loading lives outside the hot path)."""

    def __init__(self, *, teacher_model: Wav2Vec2Model, student_model: Wav2Vec2Model, distill_mode: str,
                 distill_layers: List[int], distill_linear_projs: nn.ModuleList, distill_loss: DistillLoss,
                 learning_rate: float, weight_decay: float, warmup_updates: int, max_updates: int, use_reg: bool,
                 reg_learning_rate: Optional[float], target_sparsity: Optional[float],
                 sparsity_warmup_updates: Optional[int], tsv_dir: Union[str, pathlib.Path] = ".",
                 train_subset: str = "train100", seconds_per_batch: float = 160.0, num_workers: int = 0):
        super().__init__()
        self.teacher_model = teacher_model
        self.student_model = student_model
        self.original_num_params = sum(p.numel() for p in teacher_model.parameters())
        assert distill_mode in ["layer2layer", "predlayer"], distill_mode
        assert len(distill_layers) == len(distill_linear_projs)
        self.distill_mode = distill_mode
        self.distill_layers = distill_layers
        self.distill_linear_projs = distill_linear_projs
        self.distill_loss = distill_loss
        self.learning_rate = learning_rate
        self.weight_decay = weight_decay
        self.warmup_updates = warmup_updates
        self.max_updates = max_updates
        self.use_reg = use_reg
        self.reg_learning_rate = reg_learning_rate
        self.target_sparsity = target_sparsity
        self.sparsity_warmup_updates = sparsity_warmup_updates
        if self.use_reg:
            self.lambda1 = nn.Parameter(torch.tensor(0.0))
            self.lambda2 = nn.Parameter(torch.tensor(0.0))
        self.tsv_dir = tsv_dir
        self.train_subset = train_subset
        self.seconds_per_batch = seconds_per_batch
        self.num_workers = num_workers
        self.global_step = 0
        self.target_sparsity_dev = None    # 0-d device view set by trainer.Trainer (stepstate block)
        self.teacher_stream = None         # side HIP stream for the teacher forward (trainer.Trainer)
        self._teacher_arena = ops.new_zero_arena()
        self.logged = {}
        # distinct projection modules (shared per group, distill.py:94-99) and the per-layer index into them
        uniq, index = [], []
        for m in distill_linear_projs:
            if distill_mode == "predlayer":
                # nn.Sequential(nn.Linear, nn.GELU) per distilled layer (distill.py:100-107), never shared
                if not (isinstance(m, nn.Sequential) and isinstance(m[0], nn.Linear) and isinstance(m[1], nn.GELU)
                        and m[1].approximate == "none"):
                    raise ValueError("predlayer distill heads must be nn.Sequential(nn.Linear, nn.GELU())")
                m = m[0]
            for j, u in enumerate(uniq):
                if u is m:
                    index.append(j)
                    break
            else:
                uniq.append(m)
                index.append(len(uniq) - 1)
        self._proj_uniq = uniq
        self._proj_index = index

    # ---- LightningModule surface ------------------------------------------
    def log_dict(self, d, **kw):
        # detached: a logged loss must not keep the step's autograd graph (and its AccumulateGrad
        # nodes, bound to the stream they were created on) alive into the next step / a graph capture
        self.logged.update({k: v.detach() if torch.is_tensor(v) else v for k, v in d.items()})

    def configure_optimizers(self, clip_norm: Optional[float] = None):
        main_params = [p for n, p in self.student_model.named_parameters() if "log_alpha" not in n and p.requires_grad]
        main_params.extend(list(self.distill_linear_projs.parameters()))
        seen, mp = set(), []
        for p in main_params:
            if id(p) not in seen:
                seen.add(id(p))
                mp.append(p)
        pgs = [{"params": mp, "lr": self.learning_rate, "weight_decay": self.weight_decay, "name": "main_params"}]
        if self.use_reg:
            pgs.extend([
                {"params": [p for n, p in self.student_model.named_parameters() if "log_alpha" in n],
                 "lr": self.reg_learning_rate, "weight_decay": 0.0, "name": "log_alpha"},
                {"params": [self.lambda1, self.lambda2], "lr": -self.reg_learning_rate, "weight_decay": 0.0,
                 "name": "lambda"},
            ])
        optimizer = FusedAdamW(pgs, max_grad_norm=clip_norm)
        lr_scheduler = LinearDecayLRScheduler(optimizer, warmup_updates=self.warmup_updates,
                                              max_updates=self.max_updates)
        return {"optimizer": optimizer, "lr_scheduler": {"scheduler": lr_scheduler, "interval": "step"}}

    def _get_target_sparsity(self):
        if self.global_step >= self.sparsity_warmup_updates:
            return self.target_sparsity
        return self.target_sparsity * (self.global_step / self.sparsity_warmup_updates)

    # ---- the step in three phases (trainer.Trainer captures them as separate HIP graphs) -------------------------
    def teacher_layers(self, waveforms, lengths):
        """The frozen teacher's distilled hidden states (no autograd) on the current stream."""
        with torch.no_grad():
            teacher_hiddens, _ = self.teacher_model.extract_features(waveforms, lengths)
            return [teacher_hiddens[idx] for idx in self.distill_layers]

    def student_layers(self, waveforms, lengths):
        """The student's hidden states the distill loss reads, per distilled layer."""
        student_hiddens, _ = self.student_model.extract_features(waveforms, lengths)
        if self.distill_mode == "layer2layer":
            return [student_hiddens[idx] for idx in self.distill_layers]
        if self.distill_mode == "predlayer":
            # lightning.py:259-260: every head projects the LAST student hidden state
            return [student_hiddens[-1]] * len(self.distill_layers)
        raise ValueError(f"Invalid distill mode: {self.distill_mode}")

    def _step(self, batch, batch_idx, mode):
        waveforms, lengths = batch
        self.teacher_model.eval()
        side = self.teacher_stream if waveforms.is_cuda else None
        from . import kernels as K
        # while the two forwards share the GPU, GEMMs take one tile per block (no persistent grids)
        shared = K.shared_gpu() if side is not None else contextlib.nullcontext()
        # DPH_TEACHER_ORDER=after (A/B): record the teacher branch after the student forward instead of before it
        # (a captured graph launches its nodes in recording order)
        after = side is not None and _TEACHER_AFTER
        with shared:
            if after:
                main = torch.cuda.current_stream()
                side.wait_stream(main)
                s_layers = self.student_layers(waveforms, lengths)
            if side is not None:
                # the frozen teacher runs on its own HIP stream, concurrently with the student forward: its
                # kernels fill the CUs the student's GEMM tile rounds and latency-bound launches leave idle
                # (forked / joined with stream waits, so a HIP-graph capture records both branches)
                main = torch.cuda.current_stream()
                if not after:
                    side.wait_stream(main)
                with torch.cuda.stream(side), ops.private_zero_arena(self._teacher_arena):
                    t_layers = self.teacher_layers(waveforms, lengths)
            else:
                t_layers = self.teacher_layers(waveforms, lengths)
            if not after:
                s_layers = self.student_layers(waveforms, lengths)
        if side is not None:
            main.wait_stream(side)
            for t in t_layers:
                t.record_stream(main)
        return self.loss_from_layers(s_layers, t_layers, mode)

    def loss_from_layers(self, s_layers, t_layers, mode):
        """Projections + DistillLoss + the sparsity Lagrangian on the phases' hidden states; logs the terms."""
        B, T, Ds = s_layers[0].shape
        cfg = dict(self.distill_loss.cfg(), L=len(s_layers), P=len(self._proj_uniq), B=B, T=T,
                   proj_index=self._proj_index)
        if self.distill_mode == "predlayer":
            cfg.update(head_act="gelu", shared_input=True)
        pw = []
        for m in self._proj_uniq:
            pw += [m.weight, m.bias]
        loss_distill, loss_mse, loss_l1, loss_cos = ops.DistillProjLossFn.apply(
            cfg, *[h.reshape(B * T, Ds) for h in s_layers], *pw,
            *[h.reshape(B * T, -1) for h in t_layers])
        if self.use_reg:
            cur_target_sparsity = self._get_target_sparsity()
            # the trainer keeps the target in its per-step device block (HIP-graph replays read it there)
            tgt = cur_target_sparsity if self.target_sparsity_dev is None else self.target_sparsity_dev
            # (lightning.py:221-229 in one kernel pair: ops.RegLossFn)
            loss, loss_reg, cur_expected_sparsity = ops.RegLossFn.apply(
                loss_distill, self.student_model.get_num_params(), self.lambda1, self.lambda2, tgt,
                float(self.original_num_params))
            cur_target_sparsity = tgt
        else:
            loss_reg = 0
            loss = loss_distill
        # the batched gate launch's expected #params belongs to this step only (a later get_num_params() must
        # recompute it, not return a tensor whose graph this step's backward consumes)
        self.student_model._bank_num = None
        self.log_dict({f"{mode}_loss": loss, f"{mode}_loss_distill": loss_distill, f"{mode}_loss_mse": loss_mse,
                       f"{mode}_loss_l1": loss_l1, f"{mode}_loss_cos": loss_cos, f"{mode}_loss_reg": loss_reg})
        if mode == "train" and self.use_reg:
            self.log_dict({"sparsity_expected": cur_expected_sparsity, "sparsity_target": cur_target_sparsity,
                           "lambda1": self.lambda1, "lambda2": self.lambda2})
        return loss

    def training_step(self, batch, batch_idx):
        return self._step(batch, batch_idx, mode="train")

    def validation_step(self, batch, batch_idx):
        return self._step(batch, batch_idx, mode="valid")
