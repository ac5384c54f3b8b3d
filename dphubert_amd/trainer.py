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
import time
import warnings
from typing import List, Optional

import torch
import torch.distributed as dist
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


# ---- weight-gradient group plan at world size > 1 ---------------------------------------------------------------
# Measured on one MI355X (profiles/r3_s29 kernel trace, one replayed step at B = 16 x 10 s = 7984 frames, HuBERT-Base
# with 7 087 872 parameters per encoder layer): the encoder backward without its weight gradients 4.2 ms for 12 layers;
# the grouped weight-gradient GEMMs 2.0 ms for 12 layers at 12 per launch, +0.30 / +0.46 / +0.49 / +1.39 ms at groups
# of 6 / 4 / 3 / 1 (profiles/r3_s26_*, r3_s27_*); the conv-frontend backward (pos-conv .. conv0) 3.9 ms.
WG_FRAMES = 7984
WG_LAYER_PARAMS = 7087872
WG_T_LAYER_MS = 4.2 / 12
WG_WGRAD_MS = {1: 3.39, 2: 2.9, 3: 2.49, 4: 2.46, 6: 2.30, 8: 2.2, 12: 2.0, 16: 2.0}   # per 12 layers, by group
WG_FRONTEND_MS = 3.9
XGMI_BUS_GBPS = 150.0   # ring all-reduce bus bandwidth of one xGMI ring (382 MB in ~4.4 ms at N = 8)


def grad_ready_times(model, frames: float, group: int, proj_params=()):
    """Predicted gradient-ready time (ms from the start of the encoder backward) of every student parameter with the
    encoder layers' weight gradients launched ``group`` layers at a time (ops.grouped_wgrads, flushed at the
    encoder's end too), from the measured per-layer costs above scaled by the frames and by each layer's parameter
    count.  Returns (ready {id(param): ms}, encoder end, backward end)."""
    sc = frames / WG_FRAMES
    layers = list(model.encoder.transformer.layers)
    L = len(layers)
    wg = WG_WGRAD_MS[max(k for k in WG_WGRAD_MS if k <= max(1, group))] / 12.0
    ready = {}
    t, queue = 0.0, []
    for li in reversed(range(L)):
        lay = layers[li]
        r = sum(p.numel() for n, p in lay.named_parameters() if "log_alpha" not in n) / WG_LAYER_PARAMS
        t += WG_T_LAYER_MS * sc * r
        deferred = []
        for n, p in lay.named_parameters():
            if "log_alpha" in n:
                continue
            if p.dim() == 2 and ("attention" in n or "feed_forward" in n):
                deferred.append(p)
            else:
                ready[id(p)] = t
        queue.append((r, deferred))
        if len(queue) >= group or li == 0:
            t += sum(wg * sc * rr for rr, _ in queue)
            for _, ds in queue:
                for p in ds:
                    ready[id(p)] = t
            queue = []
    t_enc = t
    t_end = t_enc + WG_FRONTEND_MS * sc
    for n, p in model.named_parameters():
        if id(p) in ready:
            continue
        # encoder-level (pos-conv, its LayerNorm, feature projection): early in the frontend window; conv stack,
        # HardConcrete logits (one bank backward at the end): at its end
        early = n.startswith("encoder.") and "log_alpha" not in n
        ready[id(p)] = t_enc + 0.1 * WG_FRONTEND_MS * sc if early else t_end
    for p in proj_params:
        ready[id(p)] = 0.0
    return ready, t_enc, t_end


def wgrad_group_timeline(model, buckets, world: int, frames: float, group: int, bus_gbps: float = XGMI_BUS_GBPS,
                         comm_bytes: int = 4, proj_params=()):
    """Predicted backward of one optimizer step (grad_ready_times): each bucket's ring all-reduce -- 2 (N-1)/N x its
    bytes at ``bus_gbps`` -- starts when its last gradient is ready and after the previous collective (one RCCL
    stream).  Returns (compute end, last collective's end) in ms."""
    ready, _, t_end = grad_ready_times(model, frames, group, proj_params)
    comm_end = 0.0
    f = 2.0 * (world - 1) / world
    for rt, n in sorted((max(ready.get(id(p), t_end) for p in b), sum(p.numel() for p in b)) for b in buckets):
        comm_end = max(comm_end, rt) + f * n * comm_bytes / (bus_gbps * 1e6)
    return t_end, comm_end


def grad_ready_order(module, params):
    """``params`` in predicted gradient-ready order (grad_ready_times at the bench shape, B = 16 x 10 s): the
    buckets then fill in the order the backward produces them -- distill projections first, encoder layers last to
    first, the frontend, and the HardConcrete logits and Lagrange multipliers (whose gradients land at the very end
    of the backward) in the last bucket instead of the first."""
    proj = list(module.distill_linear_projs.parameters())
    ready, _, t_end = grad_ready_times(module.student_model, WG_FRAMES, 12, proj)
    idx = {id(p): i for i, p in enumerate(params)}
    return sorted(params, key=lambda p: (ready.get(id(p), t_end + 1.0), idx[id(p)]))


def plan_wgrad_group(model, buckets, world: int, frames: float, bus_gbps: float = XGMI_BUS_GBPS,
                     comm_bytes: int = 4, proj_params=()) -> int:
    """The group size (layers per grouped weight-gradient launch) that minimises the predicted step end
    max(compute end, last collective end) of wgrad_group_timeline; the largest group on ties and at world size 1."""
    from . import _lib
    L = len(model.encoder.transformer.layers)
    cands = [g for g in sorted(WG_WGRAD_MS) if g <= min(L, _lib.GEMM_GROUP_MAX)] or [1]
    if world <= 1:
        return cands[-1]
    best, best_t = cands[-1], None
    for g in reversed(cands):
        te, ce = wgrad_group_timeline(model, buckets, world, frames, g, bus_gbps, comm_bytes, proj_params)
        t = max(te, ce)
        if best_t is None or t < best_t - 1e-9:
            best, best_t = g, t
    return best


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
        # (GradReducer fills its buckets in reverse registration order: hand it the reverse of the ready order)
        params = list(reversed(grad_ready_order(module, params)))
        self.reducer = GradReducer(params, bucket_mb=bucket_mb, groups=fused_grad_groups(module.student_model),
                                   comm_dtype=grad_dtype)
        if accum_grad < 1:
            raise ValueError("accum_grad must be >= 1")
        self.accum_grad = int(accum_grad)
        self._micro = 0
        self.graphs = bool(graphs)
        self.graph_warmup = max(1, int(graph_warmup))
        self._n_eager = 0                # eager OPTIMIZER steps so far
        # host seconds in the step-scalar upload and in hipGraphLaunch (bench.py host_enqueue_ms)
        self.host_s = {"upload": 0.0, "replay": 0.0, "replays": 0}
        self._graphs = {}                # (zero, final) -> (graph, static loss) or, split, ((graph A, graph B), loss)
        self._pool = None
        # split capture (DPH_GRAPH_SPLIT, default on with the teacher stream): the teacher forward is its own graph
        # replayed on the side stream, the student step two graphs on the main stream (A: forward, B: loss +
        # backward + all-reduce + AdamW) joined by a host-issued stream wait between them.  One graph with the
        # fork / join inside made hipGraphLaunch cost 5.9-11.3 ms of host time per step (its parallel branches are
        # launched node by node) against 0.3 ms for a single-stream graph (profiles/r6_s1_host_enqueue_ab.txt)
        self._split = os.environ.get("DPH_GRAPH_SPLIT", "1") != "0"
        self._tgraph = None              # (teacher graph, its static distilled hiddens, its private pool)
        self._prof_graph = None
        self._static = None
        self._prof_loss = None
        self._prof = None
        self._logged_of = {}             # id(graph) -> the module.logged dict its capture produced
        self._ffn_at = None              # global step of the last FFN compaction decision
        self._eager_until = 0            # optimizer steps before this global step run eagerly (after a layout change)
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
        # 20.67 ungrouped, profiles/r3_s27_*) (ops.grouped_wgrads; DPH_WGRAD_GROUP=1 keeps one launch per layer).
        # At world size > 1 the group is planned at the first step from the measured backward costs against the
        # buckets' all-reduce time over xGMI (plan_wgrad_group; DPH_XGMI_BUS_GBPS overrides the link rate), unless
        # DPH_WGRAD_GROUP fixes it.
        env_group = os.environ.get("DPH_WGRAD_GROUP")
        self.wgrad_group = int(env_group) if env_group else 12
        self._plan_group = env_group is None and self.reducer.world > 1
        self.wgrad_plan = None
        # replicas start from rank 0's parameters and buffers (torch DDP broadcasts at construction, distill.py:41)
        if self.reducer.world > 1:
            from .ddp import broadcast_module
            broadcast_module(module, process_group=self.reducer.group)

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
        self._backward_and_update(loss, final)
        return loss

    def _backward_and_update(self, loss, final: bool):
        # backward seeded with a persistent 1/accum_grad scalar: no ones_like fill / division launch per step
        seed = getattr(self, "_grad_seed", None)
        if seed is None or seed.device != loss.device:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("Trainer: the backward seed must exist before a graph capture")
            seed = self._grad_seed = torch.full((), 1.0 / self.accum_grad, dtype=loss.dtype, device=loss.device)
        with ops.wgrad_overlap(self._wgrad_stream), ops.grouped_wgrads(self.wgrad_group), ops.deferred_reductions():
            loss.backward(seed)
        if final:
            self.reducer.finish()
            self.optimizer.launch()

    def _capture(self, zero: bool, final: bool, prof=None):
        """Record one (micro-)step into a HIP graph (nothing executes during capture)."""
        from .kernels import LaunchProfiler
        ops.reset_zero_arena()           # zero-filled scratch must be allocated (and filled) inside the graph
        g = torch.cuda.CUDAGraph()
        try:
            if prof is not None:
                prof.__enter__()         # GEMM brackets + the non-GEMM span hook (kernels.SPAN_WORK)
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
            if prof is not None:
                prof.__exit__(None, None, None)
            ops.reset_zero_arena()
        if self._pool is None and prof is None:
            self._pool = g.pool()
        # the logged terms of this graph are the tensors its capture wrote: a replay of THIS graph refreshes them
        self._logged_of[id(g)] = dict(self.module.logged)
        return g, loss

    def _capture_split(self, zero: bool, final: bool):
        """Split capture (see __init__): the teacher graph once (its own memory pool: it replays concurrently with
        graph A), then graphs A and B of this (zero, final) kind in the shared pool, A before B (replay order)."""
        m = self.module
        side = m.teacher_stream
        from . import kernels as K
        ops.reset_zero_arena()
        try:
            if self._tgraph is None:
                m.teacher_model.eval()
                gt = torch.cuda.CUDAGraph()
                side.wait_stream(torch.cuda.current_stream())
                with K.shared_gpu(), ops.private_zero_arena(m._teacher_arena), \
                        torch.cuda.graph(gt, stream=side, capture_error_mode="thread_local"):
                    t_layers = m.teacher_layers(*self._static)
                torch.cuda.current_stream().wait_stream(side)
                self._tgraph = (gt, t_layers, gt.pool())
            t_layers = self._tgraph[1]
            ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(ga, pool=self._pool, capture_error_mode="thread_local"):
                self.reducer.prepare(zero=zero, sync=final)
                with K.shared_gpu():
                    s_layers = m.student_layers(*self._static)
            if self._pool is None:
                self._pool = ga.pool()
            with torch.cuda.graph(gb, pool=self._pool, capture_error_mode="thread_local"):
                loss = m.loss_from_layers(s_layers, t_layers, "train")
                self._backward_and_update(loss, final)
        finally:
            ops.reset_zero_arena()
        self._logged_of[id(gb)] = dict(m.logged)
        return (ga, gb), loss

    def _replay_split(self, graphs):
        ga, gb = graphs
        main, side = torch.cuda.current_stream(), self.module.teacher_stream
        side.wait_stream(main)          # this step's static input is written; the last step's loss has read t_layers
        with torch.cuda.stream(side):
            self._tgraph[0].replay()
        ga.replay()
        main.wait_stream(side)
        gb.replay()
        return gb

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

    def _drop_graphs(self):
        """Forget every captured graph AND their shared memory pool: the pool dies with its last graph, so a later
        capture into the stale pool handle trips the caching allocator (use_count assert); the next capture
        starts a new one."""
        self._graphs = {}
        self._tgraph = None
        self._prof_graph = None
        self._prof_loss = None
        self._logged_of = {}
        self._pool = None

    def verify_replicas(self):
        """Raise if any parameter / buffer differs across ranks (after a checkpoint load: cli --resume_checkpoint)."""
        from .ddp import verify_replicas
        verify_replicas(self.module, process_group=self.reducer.group)

    def _plan(self, batch):
        """World size > 1: the weight-gradient group from the step's frames (B x ~S / 320) and the bucket layout.

        Every rank must plan the SAME group: the group decides when the held-back encoder weight gradients land,
        hence the order in which buckets become ready and their collectives are issued; ranks issuing buckets in
        different orders would pair different buffers in one all-reduce (a hang, or gradients summed across the
        wrong buckets).  The bucketed train loader gives each rank its own padded length, so the plan runs on the
        largest frame count over the ranks (one MAX all-reduce of a scalar, once)."""
        self._plan_group = False
        frames = batch[0].shape[0] * batch[0].shape[1] / 320.0
        if self.reducer.world > 1 and dist.is_initialized():
            dev = batch[0].device if self.reducer.backend == "nccl" else torch.device("cpu")
            t = torch.tensor([frames], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.reducer.group)
            frames = float(t.item())
        proj = list(self.module.distill_linear_projs.parameters())
        bus = float(os.environ.get("DPH_XGMI_BUS_GBPS", XGMI_BUS_GBPS))
        cb = 2 if self.reducer.comm_dtype == torch.bfloat16 else 4
        self.wgrad_group = plan_wgrad_group(self.module.student_model, self.reducer.buckets, self.reducer.world,
                                            frames, bus, cb, proj)
        self.wgrad_plan = {"group": self.wgrad_group, "world": self.reducer.world, "frames": frames, "bus_gbps": bus,
                           "timeline_ms": wgrad_group_timeline(self.module.student_model, self.reducer.buckets,
                                                               self.reducer.world, frames, self.wgrad_group, bus, cb,
                                                               proj)}

    # ---- one step ----------------------------------------------------------------------------
    def step(self, batch, profiled: bool = False):
        m = self.module
        m.train()
        if self._plan_group:
            self._plan(batch)
        # FFN compaction policy: at the first step and every FFN_COMPACT_EVERY optimizer steps after it, eager or
        # replayed alike (one host read of the gates' expected counts: not on every eager step)
        if self._micro == 0 and (self._ffn_at is None or m.global_step - self._ffn_at >= self.FFN_COMPACT_EVERY):
            self._ffn_at = m.global_step
            if self.refresh_ffn_compaction() and self._graphs:
                # stale graphs: this optimizer step runs eagerly in the new FFN layouts (their packed buffers and
                # cached images are built outside any capture), the next one recaptures
                self._drop_graphs()
                self._eager_until = m.global_step + 1
        dev = batch[0].device
        zero = self._micro == 0
        final = self._micro + 1 == self.accum_grad
        adam_step = self.optimizer.begin_step() if final else self.optimizer._step + 1
        t_up = time.perf_counter()
        self._upload(dev, adam_step)
        self.host_s["upload"] += time.perf_counter() - t_up
        loss = None
        if self.graphs and self._n_eager >= self.graph_warmup and m.global_step >= self._eager_until:
            self._set_static(batch)
            key = (zero, final)
            split = self._split and m.teacher_stream is not None
            if key not in self._graphs:
                try:
                    self._graphs[key] = self._capture_split(zero, final) if split else self._capture(zero, final)
                except Exception as e:  # noqa: BLE001 -- uncapturable op: stay eager
                    warnings.warn(f"HIP graph capture failed, running eagerly: {e!r}")
                    self.graphs = False
                    self._drop_graphs()
            if key in self._graphs:
                if profiled and final and self._prof_graph is not None:
                    # the profiled graph's event-record nodes refer to the profiler's events (LaunchProfiler.events)
                    if self._prof is None or not self._prof.events:
                        raise RuntimeError("profiled graph without its LaunchProfiler: its events would be freed")
                    g, loss = self._prof_graph, self._prof_loss
                else:
                    g, loss = self._graphs[key]
                t_rp = time.perf_counter()
                if isinstance(g, tuple):
                    g = self._replay_split(g)
                else:
                    g.replay()
                self.host_s["replay"] += time.perf_counter() - t_rp
                self.host_s["replays"] += 1
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
