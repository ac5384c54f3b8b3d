"""Training-loop glue: builds the distill.py objects and runs one optimizer step.

Mirrors what PyTorch-Lightning did around ``DistillModule`` in the reference
(distill.py:29-144, final_distill.py:24-128): teacher (frozen) + student
(+ HardConcrete units) from ``{'state_dict','config'}`` checkpoints or from
seeded weights, identity-initialised per-group distill projections
(distill.py:24-26, 86-99), ``configure_optimizers`` (AdamW groups +
LinearDecayLR), gradient clipping, and the data-parallel all-reduce
(``dphubert_amd.ddp.GradReducer`` over RCCL).

``Trainer(graphs=True)`` replays the whole optimizer step (teacher + student forward, backward, the
gradient all-reduce, clip + AdamW) as ONE captured HIP graph after ``graph_warmup`` eager steps:
the per-step scalars (RNG epoch, learning rates, AdamW step, target sparsity) live in a device block
that the host refreshes before every step (``stepstate.StepScalars``), so replays follow the
reference schedule exactly while the host does ~50 us of work per step instead of enqueuing
~1000 kernels through Python.
"""

import copy
import os
import warnings
from typing import List, Optional

import torch
import torch.nn as nn

from . import ops
from .ddp import GradReducer
from .lightning import DistillLoss, DistillModule
from .stepstate import step_scalars
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
    """One process per GPU; call ``step(batch)`` per micro-batch (optimizer update every
    ``accum_grad`` calls).

    ``graphs=True``: the first ``graph_warmup`` optimizer steps run eagerly (they build the optimizer state,
    the gradient buckets and every cached GEMM image); after that every micro-step replays a captured HIP
    graph of its kind -- (first micro-step: zero the buckets) x (final micro-step: all-reduce, clip, AdamW);
    one graph when ``accum_grad`` is 1, three when it is > 2 (run_large.sh:54's ``--accum_grad 3``) -- each
    captured the first time it is needed, all sharing one memory pool.  Every micro-step copies its batch into
    the graphs' static input buffers, so batches must keep one shape.  If a capture fails (an op on the path
    that cannot be captured) the trainer warns and stays eager.
    """

    def __init__(self, module: DistillModule, clip_norm: float = 10.0, bucket_mb: float = 64.0,
                 accum_grad: int = 1, graphs: bool = False, graph_warmup: int = 2, grad_dtype=torch.float32):
        self.module = module
        opt = module.configure_optimizers(clip_norm=clip_norm)
        self.optimizer = opt["optimizer"]
        self.scheduler = opt["lr_scheduler"]["scheduler"]
        params = [p for g in self.optimizer.param_groups for p in g["params"]]
        self.reducer = GradReducer(params, bucket_mb=bucket_mb, groups=fused_grad_groups(module.student_model),
                                   comm_dtype=grad_dtype)
        if accum_grad < 1:
            raise ValueError("accum_grad must be >= 1")
        self.accum_grad = int(accum_grad)
        self._micro = 0
        self.graphs = bool(graphs)
        self.graph_warmup = max(1, int(graph_warmup))
        self._n_eager = 0                # eager OPTIMIZER steps so far
        self._graphs = {}                # (zero, final) -> (graph, static loss)
        self._pool = None
        self._prof_graph = None
        self._static = None
        self._prof_loss = None
        self._prof = None
        self._logged_of = {}             # id(graph) -> the module.logged dict its capture produced
        self.scalars = None
        # teacher forward on a side stream (DPH_TEACHER_STREAM=0 keeps one stream)
        if os.environ.get("DPH_TEACHER_STREAM", "1") != "0" and torch.cuda.is_available() and \
                next(module.parameters()).is_cuda:
            module.teacher_stream = torch.cuda.Stream()
        # weight-gradient GEMMs on a side stream during the backward, opt-in (DPH_WGRAD_STREAM=1): measured
        # 22.98 / 23.44 / 23.16 ms per step (conv frontend only / every layer / every layer with persistent
        # main-stream grids) against 22.95 ms on one stream -- the backward already keeps the CUs busy
        self._wgrad_stream = None
        if os.environ.get("DPH_WGRAD_STREAM", "0") == "1" and torch.cuda.is_available() and \
                next(module.parameters()).is_cuda:
            self._wgrad_stream = torch.cuda.Stream()
        # encoder-layer weight gradients launched this many layers at a time as one grouped GEMM (12: the whole
        # HuBERT-Base encoder in one launch per layer kind, 19.28 ms per step against 19.58 at 6, 19.74 at 4 and
        # 20.67 ungrouped, profiles/r3_s27_*; the buckets' collectives then overlap the conv-frontend backward)
        # (ops.grouped_wgrads; DPH_WGRAD_GROUP=1 keeps one launch per layer)
        self.wgrad_group = int(os.environ.get("DPH_WGRAD_GROUP", "12"))

    @property
    def _graph(self):
        """The graph of the final micro-step (the whole optimizer step when accum_grad is 1), or None."""
        g = self._graphs.get((self.accum_grad == 1, True))
        return g[0] if g is not None else None

    @_graph.setter
    def _graph(self, value):
        if value is None:
            self._graphs = {}
        else:
            raise AttributeError("graphs are captured by Trainer.step")

    # ---- per-step device scalars -------------------------------------------------------------
    def _bind_scalars(self, device):
        if self.scalars is None:
            self.scalars = step_scalars(device)
            self.optimizer.dyn_ptr = self.scalars.adam_dyn_ptr
            self.module.target_sparsity_dev = self.scalars.target_sparsity
        return self.scalars

    def _upload(self, device, adam_step: int):
        m = self.module
        tgt = m._get_target_sparsity() if m.use_reg else 0.0
        self._bind_scalars(device).upload(target_sparsity=tgt, adam_groups=self.optimizer.param_groups,
                                          adam_step=adam_step)

    # ---- the GPU half of one (micro-)step: no host sync, capturable ---------------------------
    def _gpu_step(self, batch, zero: bool, final: bool):
        m = self.module
        self.reducer.prepare(zero=zero, sync=final)
        loss = m.training_step(batch, 0)
        # backward seeded with a persistent 1/accum_grad scalar: no ones_like fill / division launch per step
        seed = getattr(self, "_grad_seed", None)
        if seed is None or seed.device != loss.device:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("Trainer: the backward seed must exist before a graph capture")
            seed = self._grad_seed = torch.full((), 1.0 / self.accum_grad, dtype=loss.dtype, device=loss.device)
        with ops.wgrad_overlap(self._wgrad_stream), ops.grouped_wgrads(self.wgrad_group):
            loss.backward(seed)
        if final:
            self.reducer.finish()
            self.optimizer.launch()
        return loss

    def _capture(self, zero: bool, final: bool, prof=None):
        """Record one (micro-)step into a HIP graph (nothing executes during capture)."""
        from .kernels import LaunchProfiler
        ops.reset_zero_arena()           # zero-filled scratch must be allocated (and filled) inside the graph
        g = torch.cuda.CUDAGraph()
        try:
            if prof is not None:
                LaunchProfiler.active = prof
            # thread_local: the process group's watchdog thread keeps polling the events of earlier (eager)
            # collectives while this thread captures; under the default "global" mode that poll is an illegal
            # call during capture and aborts the process ("operation not permitted when stream is capturing").
            # The profiled copy (a full training step whose GEMMs carry hand-added event-record nodes; bench.py
            # replays it as the LAST TIMED step) gets a private memory pool, so it can never alias a block the
            # main graph keeps using across replays.  Its loss terms are checked by bench.py and
            # tests/test_fullshape_gpu.py (a round-2 run reported L1 = -2.4e22 for it: an accumulator zeroed by
            # a memset node; the library zeroes with kernel nodes only since round 3, common.h zero_async)
            pool = None if prof is not None else self._pool
            with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
                loss = self._gpu_step(self._static, zero, final)
        finally:
            LaunchProfiler.active = None
            ops.reset_zero_arena()
        if self._pool is None and prof is None:
            self._pool = g.pool()
        # the logged terms of this graph are the tensors its capture wrote: a replay of THIS graph refreshes them
        self._logged_of[id(g)] = dict(self.module.logged)
        return g, loss

    def _set_static(self, batch):
        wave, lengths = batch
        if self._static is None:
            self._static = (wave.detach().clone(), lengths.detach().clone() if lengths is not None else None)
            return
        sw, sl = self._static
        if wave.shape != sw.shape or (lengths is None) != (sl is None):
            raise ValueError("Trainer(graphs=True): every batch must have the captured shape "
                             f"{tuple(sw.shape)} (got {tuple(wave.shape)})")
        if lengths is not None:
            # normalize_waveform crops the batch to max(lengths) (model.py:96-103); a captured graph replays the
            # crop of its capture, so a batch with another max(lengths) cannot be replayed (host check: one
            # small device read per step, only for models that normalize)
            for mdl in (self.module.teacher_model, self.module.student_model):
                hint = getattr(mdl, "_lmax_hint", None) if getattr(mdl, "normalize_waveform", False) else None
                if hint is not None and int(lengths.max()) != hint[1]:
                    raise ValueError(f"Trainer(graphs=True): max(lengths) = {int(lengths.max())} differs from the "
                                     f"captured crop length {hint[1]} (normalize_waveform)")
        sw.copy_(wave)
        if lengths is not None:
            sl.copy_(lengths)

    def prepare_profiled_step(self, prof):
        """Capture a second graph of the final micro-step whose GEMM launches are bracketed by timing events
        (bench.py's live roofline); ``step(batch, profiled=True)`` replays it."""
        if self._graph is None:
            raise RuntimeError("prepare_profiled_step needs the main graph (run the warm-up steps first)")
        # the profiled copy runs the teacher on the main stream: with the side stream, parallel graph branches
        # interleave between an event pair and the pair no longer brackets one kernel (live 75 us vs 58 us in
        # the rocprof trace for the same launches)
        # the graph's event-record nodes refer to the profiler's hipEvents: keep it (and them) alive as long as
        # the graph can be replayed (a collected profiler destroys its events -> replay faults on the host)
        self._prof = prof
        side, self.module.teacher_stream = self.module.teacher_stream, None
        wside, self._wgrad_stream = self._wgrad_stream, None
        try:
            self._prof_graph, self._prof_loss = self._capture(self.accum_grad == 1, True, prof)
        finally:
            self.module.teacher_stream = side
            self._wgrad_stream = wside

    # ---- FFN-unit compaction policy ------------------------------------------------------------
    FFN_COMPACT_MIN_ZERO = 0.3       # expected fraction of exactly-zero FFN units from which the packed FFN pays
    FFN_COMPACT_EVERY = 500          # optimizer steps between re-evaluations under graph replay

    def refresh_ffn_compaction(self) -> bool:
        """Per FFN intermediate HardConcrete gate: run the layer's FFN GEMMs over the active units only
        (ops._ffn_forward) when the expected fraction of exactly-zero units, 1 - l0_norm / n (hardconcrete.py:62-65:
        P(mask != 0) = sigmoid(log_alpha - beta log(-l / r))), is >= FFN_COMPACT_MIN_ZERO.  One host read of
        the expected counts.  Returns whether any gate changed its mode (captured graphs are then stale)."""
        from .wav2vec2.hardconcrete import HardConcrete
        mods = [mod for name, mod in self.module.student_model.named_modules()
                if isinstance(mod, HardConcrete) and name.endswith("hard_concrete_for_intermediate")]
        if not mods:
            return False
        with torch.no_grad():
            nz = torch.stack([mod.l0_norm() for mod in mods]).float().cpu().tolist()
        changed = False
        for mod, k in zip(mods, nz):
            flag = 1.0 - k / mod.n_in >= self.FFN_COMPACT_MIN_ZERO
            if bool(getattr(mod, "dph_compact", False)) != flag:
                mod.dph_compact = flag
                changed = True
        return changed

    # ---- one step ----------------------------------------------------------------------------
    def step(self, batch, profiled: bool = False):
        m = self.module
        m.train()
        if self._micro == 0 and (not self._graphs or m.global_step % self.FFN_COMPACT_EVERY == 0):
            if self.refresh_ffn_compaction() and self._graphs:
                self._graphs = {}            # recaptured at this step with the new FFN layouts
                self._prof_graph = None
        dev = batch[0].device
        zero = self._micro == 0
        final = self._micro + 1 == self.accum_grad
        adam_step = self.optimizer.begin_step() if final else self.optimizer._step + 1
        self._upload(dev, adam_step)
        loss = None
        if self.graphs and self._n_eager >= self.graph_warmup:
            self._set_static(batch)
            key = (zero, final)
            if key not in self._graphs:
                try:
                    self._graphs[key] = self._capture(zero, final)
                except Exception as e:  # noqa: BLE001 -- uncapturable op: stay eager
                    warnings.warn(f"HIP graph capture failed, running eagerly: {e!r}")
                    self.graphs = False
                    self._graphs = {}
            if key in self._graphs:
                if profiled and final and self._prof_graph is not None:
                    g, loss = self._prof_graph, self._prof_loss
                else:
                    g, loss = self._graphs[key]
                g.replay()
                m.logged = dict(self._logged_of[id(g)])
        if loss is None:
            loss = self._gpu_step(batch, zero, final)
            if final:
                self._n_eager += 1
        if not final:
            self._micro += 1
            return loss.detach()
        self._micro = 0
        loss = loss.detach()
        self.scheduler.step()
        if not self._graphs:
            for g in self.optimizer.param_groups:
                for p in g["params"]:
                    p.grad = None
        m.global_step += 1
        return loss
