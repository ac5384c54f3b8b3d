"""DPHuBERT distill-step benchmark on MI355X (see BASELINE.json / SURVEY.md 8(d)).

One step = the reference's distill.py training step (lightning.py:245-296 + the
Lightning loop): frozen teacher forward (eval), student forward in training mode
(dropout, HardConcrete conv/head/interm masks sampled), per-group projections,
L1 + cosine distillation loss, Lagrangian expected-sparsity regulariser,
backward, RCCL gradient all-reduce (N > 1), grad-norm clip (10) and AdamW,
on synthetic 10 s / 16 kHz waveforms, B utterances per GPU (default 16 =
run.sh's 160 s per GPU), HuBERT-Base teacher+student with seeded weights.

Prints ONE JSON line on rank 0.  Launch N > 1 with
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
      --master-port P bench.py --gpus N
"""

import argparse
import copy
import csv
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import torch
import torch.distributed as dist

FLOP_PER_UTT_BASE = 599.6e9      # teacher fwd + 3 x (student fwd + projections), 10 s utterance
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dphubert_amd.perfmodel import HBM_PEAK_GBPS, MFMA_PEAK_TFLOPS, forward_flops, step_flops_per_utt  # noqa: E402,F401,E501


def workload(args):
    """(teacher config, student config or None, DistillModule kwargs, description) of the benched step."""
    from dphubert_amd.synthetic import HUBERT_BASE_CONFIG, WAVLM_BASE_CONFIG, WAV2VEC2_LARGE_CONFIG
    tcfg = {"wavlm-base": WAVLM_BASE_CONFIG, "large": WAV2VEC2_LARGE_CONFIG}.get(args.model, HUBERT_BASE_CONFIG)
    layers = "0.4,8,12,16,20,24" if args.model == "large" else "0.4,8,12"       # run_large.sh:13 / run.sh:21
    if args.student == "pruned":
        # final_distill.py (run.sh:95-115): the pruned student (prune() of a 0.75-sparsity student, ~23.6 M
        # params), no HardConcrete units, no regulariser (final_distill.py:115), lr 1e-4
        from dphubert_amd.synthetic import pruned_student
        scfg, ssd = pruned_student(tcfg, seed=0)
        kw = dict(student_config=scfg, student_state=ssd, use_reg=False, learning_rate=1e-4, warmup_updates=5000,
                  max_updates=25000)
        desc = "final_distill.py step: {fam} teacher (eval) + pruned student (train, ~23.6 M params, dropout)"
    else:
        scfg = dict(tcfg, extractor_prune_conv_channels=True, encoder_prune_attention_heads=True,
                    encoder_prune_feed_forward_intermediate=True)
        kw = dict(pruning_units="conv,head,interm", use_reg=True)
        desc = ("distill.py step: {fam} teacher (eval) + student (train, HardConcrete conv,head,interm, dropout) + "
                "L1/cos distill loss + sparsity Lagrangian + AdamW")
    return tcfg, scfg, layers, kw, desc


def trained_like_masks(student, seed: int = 0):
    """log_alpha of a prune.py student near its 0.75 target: per layer, a seeded random subset of 4 of 12 heads,
    768 of 3072 FFN units and 320 of 512 conv channels at log_alpha = +10 (sampled mask 1), the rest at -10
    (sampled s < 0, clamped to exactly 0 by hardconcrete.py:99 -- the heads the attention kernels skip)."""
    keep = {"hard_concrete_for_heads": 1 / 3, "hard_concrete_for_intermediate": 0.25, "hard_concrete": 0.625}
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, mod in student.named_modules():
            frac = keep.get(name.rsplit(".", 1)[-1])
            if frac is None or getattr(mod, "log_alpha", None) is None:
                continue
            n = mod.log_alpha.numel()
            k = max(1, round(frac * n))
            la = torch.full((n,), -10.0)
            la[torch.randperm(n, generator=g)[:k]] = 10.0
            mod.log_alpha.copy_(la.to(mod.log_alpha.device))


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cores() -> int:
    """Host cores this process may use: its CPU affinity set, bounded by the job's thread budget
    (OMP_NUM_THREADS, which the GPU box sets to this job's CPU share; os.cpu_count() there reports the
    whole machine, whose other cores belong to other jobs)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(batch: int = 2, warmup: int = 3, steps: int = 5, seconds: float = 10.0):
    """Time the fp32 CPU oracle (oracle/hubert_ref.py) on a bounded sample of the same step
    (B=2, 3 warm-up + 5 timed steps, all host cores of this job, CPU model stated)."""
    from dphubert_amd.synthetic import HUBERT_BASE_CONFIG, seeded_state_dict, synthetic_batch
    from oracle import hubert_ref as ref
    threads = host_cores()
    torch.set_num_threads(threads)
    cfg = copy.deepcopy(HUBERT_BASE_CONFIG)
    scfg = dict(cfg, extractor_prune_conv_channels=True, encoder_prune_attention_heads=True,
                encoder_prune_feed_forward_intermediate=True)
    tsd = seeded_state_dict(ref.state_dict_shapes(cfg), 0)
    ssd = seeded_state_dict(ref.state_dict_shapes(scfg), 0)
    psd = {"0.weight": torch.eye(768), "0.bias": torch.zeros(768), "1.weight": torch.eye(768),
           "1.bias": torch.zeros(768)}
    wave, lengths = synthetic_batch(batch, int(seconds * 16000))
    g = torch.Generator().manual_seed(0)
    u = {n[:-len(".log_alpha")]: torch.rand(v.shape, generator=g) * 0.98 + 0.01 for n, v in ssd.items()
         if n.endswith(".log_alpha")}
    kw = dict(teacher_sd=tsd, teacher_cfg=cfg, student_sd=ssd, student_cfg=scfg, proj_sd=psd,
              distill_layers=[0, 4, 8, 12], proj_index=[0, 1, 1, 1], wave=wave, lengths=lengths, u=u,
              lambdas=(0.0, 0.0), global_step=5000, original_num_params=94371456)
    for _ in range(warmup):
        ref.distill_step(**kw)
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        ref.distill_step(**kw)
        times.append(time.perf_counter() - t0)
    dt = sorted(times)[len(times) // 2]          # median step
    return {"value": round(batch * seconds / dt, 3), "unit": "audio-seconds/sec", "cores": threads,
            "kind": "port", "cpu_model": _cpu_model(), "median_step_s": round(dt, 3),
            "sample": f"oracle/hubert_ref.py distill_step (teacher fwd + student fwd/bwd + loss + reg, fp32, no "
                      f"optimizer), HuBERT-Base 12 layers, B={batch} x {seconds:.0f} s, median of {steps} timed steps "
                      f"after {warmup} warm-up, torch CPU {threads} threads on {_cpu_model()}"}


def pmc_traffic(args):
    """HBM bytes of every GEMM, attention and conv0 kernel variant from rocprofv3 PMC counters.

    Two child runs of this script (1 warm-up + 1 step, same workload), one counter per pass
    (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass), started before this process touches the
    GPU.  gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE is in KiB and reports
    half the bytes of wide coalesced reads -> bytes = 2 * 1024 * FETCH_SIZE; WRITE_SIZE is exact
    for 16-B stores -> bytes = 1024 * WRITE_SIZE.  Returns {kernel name: [total bytes, launches]}
    (launches of the FETCH pass; both passes run the same launches).  DPH_BENCH_PMC_DIR: keep the
    counter CSVs there (profiles/ evidence of the traffic figures).
    """
    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        raise RuntimeError("rocprofv3 not found")
    here = os.path.dirname(os.path.abspath(__file__))
    out = {}
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        for counter, scale in (("FETCH_SIZE", 2 * 1024.0), ("WRITE_SIZE", 1024.0)):
            d = os.path.join(td, counter)
            cmd = [exe, "--pmc", counter, "--kernel-include-regex", "gemm_kernel|attn_|conv0_", "-f", "csv", "-d", d,
                   "-o", "run",
                   "--", sys.executable, os.path.join(here, "bench.py"), "--steps", "1", "--warmup", "1",
                   "--no-cpu-baseline", "--no-roofline", "--traffic", "off", "--graphs", "off", "--batch", str(args.batch),
                   "--seconds", str(args.seconds), "--model", args.model, "--student", args.student]
            env = dict(os.environ, TMPDIR="/tmp")
            r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                               timeout=400)
            if r.returncode != 0:
                raise RuntimeError(f"rocprofv3 {counter} pass failed ({r.returncode}): {r.stdout[-400:]!r}")
            files = [os.path.join(dp, f) for dp, _, fs in os.walk(d) for f in fs
                     if f.endswith("counter_collection.csv")]
            if not files:
                raise RuntimeError(f"rocprofv3 {counter}: no counter_collection.csv")
            keep = os.environ.get("DPH_BENCH_PMC_DIR")
            if keep:
                os.makedirs(keep, exist_ok=True)
                shutil.copy(files[0], os.path.join(keep, f"pmc_{counter}.csv"))
            sums = {}
            for row in csv.DictReader(open(files[0])):
                if row["Counter_Name"] != counter:
                    continue
                v = sums.setdefault(row["Kernel_Name"], [0.0, 0])
                v[0] += float(row["Counter_Value"]) * scale
                v[1] += 1
            for k, (tot, n) in sums.items():
                o = out.setdefault(k, [0.0, 0])
                o[0] += tot / n          # mean bytes per launch of this counter ...
                o[1] = max(o[1], n)
    return {k: [b * n, n] for k, (b, n) in out.items()}   # ... -> total bytes over the launches


# rocprof kernel-name fragments of the launches behind each kernel_table span (kernels.SPAN_WORK labels)
SPAN_KERNELS = {
    "attn_fwd_drop": ["attn_fwd32v2_kernel<true"], "attn_fwd": ["attn_fwd32v2_kernel<false"],
    "attn_bwd_drop": ["attn_bwd_kernel<true"], "attn_bwd": ["attn_bwd_kernel<false"],
    "conv0_gn_fwd": ["conv0_gram_part_kernel", "conv0_gram_reduce", "conv0_apply_kernel<true"],
    "conv0_gn_bwd": ["conv0_gram_part_kernel", "conv0_gram_reduce", "conv0_gn_bwd_kernel", "conv0_bwd_finalize"],
}


def traffic_per_launch(traffic, frags):
    """PMC bytes per launch summed over the kernels a span launches (each fragment: launch-weighted over every
    template variant whose rocprof name contains it)."""
    if not traffic:
        return None
    tot = 0.0
    for fr in frags:
        hits = [v for k, v in traffic.items() if fr in k]
        if not hits:
            return None
        tot += sum(b for b, _ in hits) / sum(n for _, n in hits)
    return tot


def check_step(loss: float, terms, main_loss):
    """Refuse to report a throughput measured on a corrupted step: the last timed step's loss must be finite and
    its logged terms (lightning.py:277-295) self-consistent -- L1 = mean|s - t| > 0, the cosine term in [-1, 1],
    loss = distill + reg, expected sparsity in [0, 1] -- and, when the last step replayed the profiled graph, its
    loss must lie near the main graph's (the two replay the same step; the losses differ only by the step's own
    dropout / HardConcrete draws, |diff| well below 1)."""
    import math
    bad = []
    if not math.isfinite(loss):
        bad.append(f"loss {loss}")
    if terms:
        l1, cos = terms.get("train_loss_l1"), terms.get("train_loss_cos")
        dist_, reg = terms.get("train_loss_distill"), terms.get("train_loss_reg", 0.0)
        es = terms.get("sparsity_expected")
        if l1 is not None and not (0.0 < l1 < 1e3):
            bad.append(f"l1 {l1}")
        if cos is not None and not (-1.0 - 1e-5 <= cos <= 1.0 + 1e-5):
            bad.append(f"cos {cos}")
        if dist_ is not None and abs(terms.get("train_loss", loss) - (dist_ + reg)) > 1e-4 * max(1.0, abs(loss)):
            bad.append(f"loss {terms.get('train_loss')} != distill {dist_} + reg {reg}")
        if es is not None and not (-1e-6 <= es <= 1.0 + 1e-6):
            bad.append(f"expected sparsity {es}")
    if main_loss is not None and abs(loss - main_loss) > 0.5:
        bad.append(f"last step loss {loss} vs main graph {main_loss}")
    if bad:
        raise SystemExit("bench.py: the measured step is corrupted: " + "; ".join(bad))


def bucketed_batches(n: int, seconds_per_batch: float, rank: int, dev):
    """n batches shaped like distill.py's train loader (data.train_loader): 4000 synthetic utterance lengths
    uniform in 2-15.6 s (the loader's min_len / max_len), 1000 length buckets, a seconds_per_batch token
    budget, crop-to-shortest collate; n batches taken evenly over the length range (seeded)."""
    from dphubert_amd.data import BucketizeBatchSampler
    g = torch.Generator().manual_seed(2022)
    lens = torch.randint(32000, 250001, (4000,), generator=g).tolist()
    bs = BucketizeBatchSampler(lens, num_buckets=1000, max_token_count=int(seconds_per_batch * 16000),
                               min_len=32000, max_len=250000, shuffle=False)
    packs = list(bs)
    pick = [packs[int(i * (len(packs) - 1) / max(n - 1, 1))] for i in range(n)]
    perm = torch.randperm(n, generator=g).tolist()            # lengths in no particular order over the steps
    out = []
    gw = torch.Generator().manual_seed(2022 + rank)
    for k in perm:
        idx = pick[k]
        L = min(lens[i] for i in idx)
        w = 0.1 * torch.randn(len(idx), L, generator=gw)
        out.append((w.to(dev), torch.full((len(idx),), L, dtype=torch.int64).to(dev)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None,
                    help="utterances per GPU per micro-batch (default: 16 = run.sh's 160 s per GPU; 8 for --student "
                         "pruned = 640 s over 8 GPUs, SURVEY 8(d) config 4; 6 for --model large = run_large.sh's 60 s)")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--model", choices=["hubert-base", "wavlm-base", "large"], default="hubert-base",
                    help="teacher/student family (the headline metric is quoted on hubert-base; large = the "
                         "wav2vec2-Large teacher of run_large.sh:11, 24 pre-norm layers, distill layers 0.4,8,12,16,20,24)")
    ap.add_argument("--student", choices=["prune", "pruned"], default="prune",
                    help="prune: distill.py's joint distill + prune step (HardConcrete units, regulariser); pruned: "
                         "final_distill.py's step on a pruned ~23.6 M-parameter student (no HardConcrete)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--traffic", choices=["auto", "off"], default="auto",
                    help="auto: measure per-launch HBM bytes of the GEMMs with rocprofv3 PMC passes (rank 0, N=1)")
    ap.add_argument("--grad-comm", choices=["fp32", "bf16"], default="fp32",
                    help="payload of the gradient all-reduce at N > 1 (bf16: half the xGMI bytes)")
    ap.add_argument("--accum", type=int, default=1, help="micro-batches per optimizer step (a step = one micro-batch)")
    ap.add_argument("--masks", choices=["init", "trained"], default="init",
                    help="student HardConcrete log_alpha: the reference init (hardconcrete.py:70-74; the headline) or "
                         "trained-like = a prune.py student near its 0.75 target (log_alpha +-10: 4 of 12 heads, 768 of "
                         "3072 FFN units and 320 of 512 conv channels per layer kept, the rest sampled exactly 0)")
    ap.add_argument("--graphs", choices=["on", "off"], default="on",
                    help="on: replay the whole step as one captured HIP graph after the eager warm-up steps")
    ap.add_argument("--lengths", choices=["fixed", "bucketed"], default="fixed",
                    help="fixed: B x --seconds utterances (the headline); bucketed: the reference's train loader "
                         "shapes -- 2-15.6 s utterance lengths, 1000 length buckets, a 160 s token budget per "
                         "batch, crop-to-shortest collate (lightning.py:306-325) -- one new shape per step, eager")
    args = ap.parse_args()
    if args.lengths == "bucketed":
        args.graphs = "off"
    if args.batch is None:
        args.batch = 6 if args.model == "large" else (8 if args.student == "pruned" else 16)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    traffic, traffic_err = None, None
    if world == 1 and not args.no_roofline and args.traffic == "auto":
        # before this process initialises the GPU (the profiled children own it meanwhile)
        try:
            traffic = pmc_traffic(args)
        except Exception as e:  # noqa: BLE001 -- traffic is informational
            traffic_err = repr(e)[:300]
    # DPH_BENCH_BACKEND=gloo (rehearsal of the N > 1 path on one GPU: every rank on device LOCAL_RANK % count, gloo
    # collectives, eager steps -- gloo collectives cannot be captured); the scaling runs use the default, nccl = RCCL
    backend = os.environ.get("DPH_BENCH_BACKEND", "nccl")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "gloo":
            local_rank %= torch.cuda.device_count()
            args.graphs = "off"
        torch.cuda.set_device(local_rank)
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from dphubert_amd import ops
    from dphubert_amd.kernels import LaunchProfiler
    from dphubert_amd.synthetic import synthetic_batch
    from dphubert_amd.trainer import Trainer, build_distill_module

    ops.manual_seed(2022 + rank)
    tcfg, scfg, distill_layers, mkw, desc = workload(args)
    module = build_distill_module(tcfg, distill_layers=distill_layers, **mkw)
    n_student = sum(p.numel() for n, p in module.student_model.named_parameters() if "log_alpha" not in n)
    flop_utt = step_flops_per_utt(tcfg, scfg, len(module.distill_layers), int(args.seconds * 16000))
    module.global_step = 5000            # target sparsity reached (0.75)
    if args.masks == "trained":
        trained_like_masks(module.student_model)
    module = module.to(dev)
    graphs = args.graphs == "on"
    trainer = Trainer(module, clip_norm=10.0, graphs=graphs, graph_warmup=2, accum_grad=args.accum,
                      grad_dtype=torch.bfloat16 if args.grad_comm == "bf16" else torch.float32)
    samples = int(args.seconds * 16000)
    wave, lengths = synthetic_batch(args.batch, samples, seed=2022 + rank)
    batch = (wave.to(dev), lengths.to(dev))
    batches = None
    if args.lengths == "bucketed":
        batches = bucketed_batches(args.warmup + args.steps, args.batch * args.seconds, rank, dev)

    # warm-up: 2 eager steps, then (graphs) the capture + first replay
    if args.accum < 1 or args.steps < args.accum:
        raise SystemExit("--accum must be >= 1 and <= --steps")
    # warm-up in whole optimizer steps (the trainer captures its graphs after 2 eager optimizer steps)
    n_warm = max(args.warmup, 3 if graphs else 1) * args.accum
    for i in range(n_warm):
        loss = trainer.step(batch if batches is None else batches[i % len(batches)])
    torch.cuda.synchronize()
    graphed = trainer._graph is not None
    log(f"step mode: {'HIP graph replay' if graphed else 'eager'}")
    ddp_plan = None
    if world > 1:
        # the data-parallel plan of this run: buckets, the weight-gradient group planned on the MAX frame
        # count over the ranks, and the modelled window (compute end vs last collective end, ms from the start of
        # the encoder backward) at the assumed xGMI ring rate
        red = trainer.reducer
        plan = trainer.wgrad_plan or {"group": trainer.wgrad_group}
        ddp_plan = {"buckets": len(red.flat), "bucket_mb": [round(f.numel() * f.element_size() / 2 ** 20, 1)
                                                            for f in red.flat],
                    "grad_comm": args.grad_comm, "wgrad_group": plan.get("group"), "frames": plan.get("frames"),
                    "assumed_bus_gbps": plan.get("bus_gbps"),
                    "modelled_compute_end_ms": round(plan["timeline_ms"][0], 3) if "timeline_ms" in plan else None,
                    "modelled_comm_end_ms": round(plan["timeline_ms"][1], 3) if "timeline_ms" in plan else None}
        log(f"ddp plan: {json.dumps(ddp_plan)}")
    # GEMM launches of the LAST timed step are bracketed by HIP events on their launch stream (an
    # event marker costs ~3 us of GPU time, so bracketing every step would tax the headline number).
    # With graphs, that step replays a second capture of the same step whose GEMMs carry event nodes.
    # DPH_BENCH_SHAPES=1: key the profiled step's GEMM table by shape / epilogue too (diagnostics, stderr)
    by_shape = os.environ.get("DPH_BENCH_SHAPES") == "1"
    prof = LaunchProfiler(by_shape=by_shape) if (rank == 0 and not args.no_roofline) else None
    prof_mode = "timed step" if prof is not None else None
    if prof is not None and graphed:
        try:
            trainer.prepare_profiled_step(prof)
            prof_mode = "last timed step (graph replay with event nodes)"
        except Exception as e:  # noqa: BLE001 -- event nodes not capturable: profile an eager step after timing
            log(f"profiled capture unavailable ({e!r}); GEMMs are timed on an eager step after the timed region")
            prof = LaunchProfiler()
            prof_mode = "eager step right after the timed region (same kernels)"
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    # host-side accounting of the timed loop: the step-scalar ring blocks the host once it runs RING steps ahead
    # of the GPU (stepstate.StepScalars), so the loop's host time minus that blocked time is the enqueue cost
    scal = trainer._bind_scalars(dev)
    scal.wait_s = 0.0
    trainer.host_s = {"upload": 0.0, "replay": 0.0, "replays": 0}
    t0 = time.perf_counter()
    in_loop = prof is not None and prof_mode != "eager step right after the timed region (same kernels)"
    last_final = (args.steps // args.accum) * args.accum - 1    # the last micro-step that ends an optimizer step
    audio_timed = 0.0
    for i in range(args.steps):
        last = in_loop and i == last_final
        if last and not graphed:
            prof.__enter__()
        b = batch if batches is None else batches[args.warmup + i]
        audio_timed += b[0].shape[0] * b[0].shape[1] / 16000.0
        loss = trainer.step(b, profiled=last)
    t_host = time.perf_counter() - t0          # host enqueue time (GPU may still be running)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    ms = dt / args.steps * 1e3
    audio_s = world * audio_timed            # (every rank processes the same amount: shapes per rank differ)
    value = audio_s / dt
    host = {"host_loop_ms": round(t_host / args.steps * 1e3, 3),
            "host_blocked_ms": round(scal.wait_s / args.steps * 1e3, 3),
            "host_enqueue_ms": round((t_host - scal.wait_s) / args.steps * 1e3, 3),
            "host_replay_ms": round(trainer.host_s["replay"] / max(1, trainer.host_s["replays"]) * 1e3, 3),
            "host_upload_ms": round((trainer.host_s["upload"] - scal.wait_s) / args.steps * 1e3, 3)}
    log(f"host loop {host['host_loop_ms']:.2f} ms/step = enqueue {host['host_enqueue_ms']:.2f} "
        f"(hipGraphLaunch {host['host_replay_ms']:.2f}, scalar upload {host['host_upload_ms']:.3f}) + blocked on the "
        f"step-scalar ring {host['host_blocked_ms']:.2f}")
    log(f"loss {loss.item():.5f}  step {ms:.2f} ms  {value:.1f} audio-s/s  "
        f"({flop_utt * args.batch / (ms / 1e3) / 1e12:.0f} TFLOP/s algorithmic/GPU)")
    terms = {k: (float(v.float().sum()) if torch.is_tensor(v) else v)
             for k, v in getattr(trainer.module, "logged", {}).items()}
    if os.environ.get("DPH_BENCH_LOGGED") == "1":      # diagnostics: the last replayed graph's logged terms
        log(f"logged terms: {terms}")
    main_loss = None
    # (accum 1 only: with accumulation the final micro-step graph's loss output is refreshed by the next
    # optimizer step's first micro-step replay, so after the loop it no longer holds that step's loss)
    if graphed and args.accum == 1 and trainer._graphs.get((True, True)) is not None:
        main_loss = trainer._graphs[(True, True)][1].item()     # the last main-graph replay
    check_step(loss.item(), terms if (graphed or in_loop) else None, main_loss)

    fam = {"wavlm-base": "WavLM-Base", "large": "wav2vec2-Large"}.get(args.model, "HuBERT-Base")
    utts = "10s utts" if batches is None else "bucketed 2-15.6s utts, 160 s/batch"
    out = {
        "metric": f"audio-seconds/sec/node ({fam} {'final_distill' if args.student == 'pruned' else 'distill'} step, "
              f"{utts})",
        "value": round(value, 2),
        "unit": "audio-seconds/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": f"synthetic (0.1*randn 16 kHz waveforms, seeded random-init {fam} weights)",
        "config": {"workload": desc.format(fam=fam),
                   "utterances_per_gpu": args.batch, "seconds_per_utt": args.seconds,
                   "global_batch_audio_s": world * args.batch * args.seconds * args.accum,
                   "distill_layers": distill_layers, "student_params": n_student,
                   "step_gflop_per_utt": round(flop_utt / 1e9, 1),
                   "parallelism": f"dp{world}", "accum_grad": args.accum, "grad_comm": args.grad_comm,
                   "lengths": args.lengths, "masks": args.masks},
        "peak_hbm_gib": round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2),
        "step_mode": "hip_graph" if graphed else "eager",
        "host": host,
    }
    if ddp_plan is not None:
        out["ddp_plan"] = ddp_plan
    if prof is not None and not in_loop:
        torch.cuda.synchronize()
        saved, trainer._graphs = trainer._graphs, {}      # one eager step with the profiler on
        g_on = trainer.graphs
        trainer.graphs = False
        with prof:
            trainer.step(batch)
        trainer.graphs, trainer._graphs = g_on, saved
    if prof is not None:
        prof.__exit__(None, None, None)
        summ = prof.summary()
        if by_shape:
            for k, v in sorted(summ.items(), key=lambda kv: -kv[1]["ms"]):
                log(f"{v['ms']:7.3f} ms {v['launches']:4d}x {v['ms'] / v['launches'] * 1e3:7.1f} us "
                    f"{v['flops'] / v['ms'] / 1e9:6.0f} TF/s  {k}")
            agg = {}
            for k, v in summ.items():
                d = agg.setdefault(k.split(" M=")[0], {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0})
                for f in d:
                    d[f] += v[f]
            summ = agg
        top = max(summ.items(), key=lambda kv: kv[1]["ms"])
        name, d = top
        avg_ms = d["ms"] / d["launches"]
        flops_per_launch = d["flops"] / d["launches"]
        achieved = flops_per_launch / (avg_ms / 1e3) / 1e12
        all_ms = sum(v["ms"] for v in summ.values())
        all_fl = sum(v["flops"] for v in summ.values())
        tr = None
        if traffic:
            # launch-weighted over EVERY template variant of the dominant kernel (the algorithmic bytes below
            # average all of its launches too)
            hits = [v for k, v in traffic.items() if name in k]
            tr = round(sum(b for b, _ in hits) / sum(n for _, n in hits)) if hits else None
        alg_b = d["bytes"] / d["launches"]
        out["roofline"] = {"bound": "mfma", "kernel": name, "achieved": round(achieved, 1),
                           "peak": MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / MFMA_PEAK_TFLOPS, 4),
                           "traffic": tr, "traffic_unit": "bytes/launch (HBM, PMC FETCH_SIZE*2 + WRITE_SIZE)",
                           "algorithmic_bytes": round(alg_b),
                           "traffic_ratio": round(tr / alg_b, 3) if tr else None,
                           "launches_per_step": d["launches"],
                           "avg_launch_us": round(avg_ms * 1e3, 2), "flop_per_launch": flops_per_launch,
                           "all_gemm_tflops": round(all_fl / (all_ms / 1e3) / 1e12, 1),
                           "gemm_ms_per_step": round(all_ms, 3), "timed_on": prof_mode}
        if traffic_err:
            out["roofline"]["traffic_error"] = traffic_err
        log(json.dumps({k: v for k, v in summ.items()}))
        # the non-GEMM kernels of the same profiled step against their own roof: attention on the MFMA peak
        # (algorithmic FLOPs), conv0 / LayerNorm / AdamW on HBM (the bytes each launch must move once)
        table = []
        for label, d in sorted(prof.span_summary().items(), key=lambda kv: -kv[1]["ms"]):
            avg_s = d["ms"] / d["launches"] / 1e3
            per = d["work"] / d["launches"]
            if d["unit"] == "flop":
                ach, peak, unit = per / avg_s / 1e12, MFMA_PEAK_TFLOPS, "TFLOP/s"
            else:
                ach, peak, unit = per / avg_s / 1e9, HBM_PEAK_GBPS, "GB/s"
            row = {"kernel": label, "bound": "mfma" if d["unit"] == "flop" else "hbm",
                   "launches_per_step": d["launches"], "avg_launch_us": round(avg_s * 1e6, 2),
                   "work_per_launch": per, "work_unit": d["unit"], "achieved": round(ach, 1), "peak": peak,
                   "unit": unit, "frac": round(ach / peak, 4), "ms_per_step": round(d["ms"], 3)}
            if label in SPAN_KERNELS:
                tb = traffic_per_launch(traffic, SPAN_KERNELS[label])
                row["pmc_bytes_per_launch"] = round(tb) if tb else None
                if tb and d["unit"] == "byte":
                    row["traffic_ratio"] = round(tb / per, 3)
            table.append(row)
        out["kernel_table"] = table
        # north_star's bar: MFMA utilisation of masked attention + FFN over the same profiled step -- the algorithmic
        # FLOPs of every attention launch (forward Q K^T + P V, backward 2.5x) and of every FFN GEMM (FFN1 / FFN2
        # forward of teacher and student, their input and weight gradients) over the summed event-timed durations
        spans = prof.span_summary()
        attn = [v for k, v in spans.items() if k.startswith("attn_")]
        ffn = prof.role_summary().get("ffn")
        a_ms, a_fl = sum(v["ms"] for v in attn), sum(v["work"] for v in attn)
        f_ms, f_fl = (ffn["ms"], ffn["flops"]) if ffn else (0.0, 0.0)
        if a_ms + f_ms > 0:
            util = (a_fl + f_fl) / ((a_ms + f_ms) / 1e3) / 1e12 / MFMA_PEAK_TFLOPS
            out["mfma_util_attn_ffn"] = round(util, 4)
            out["mfma_util_detail"] = {
                "attention": {"ms_per_step": round(a_ms, 3), "gflop": round(a_fl / 1e9, 1),
                              "util": round(a_fl / (a_ms / 1e3) / 1e12 / MFMA_PEAK_TFLOPS, 4) if a_ms else None},
                "ffn_gemms": {"ms_per_step": round(f_ms, 3), "gflop": round(f_fl / 1e9, 1),
                              "launches": ffn["launches"] if ffn else 0,
                              "util": round(f_fl / (f_ms / 1e3) / 1e12 / MFMA_PEAK_TFLOPS, 4) if f_ms else None},
                "peak_tflops": MFMA_PEAK_TFLOPS, "timed_on": prof_mode}
    if batches is not None:
        shapes = [tuple(b[0].shape) for b in batches[args.warmup:]]
        out["config"]["batch_shapes"] = [f"{bb}x{ss / 16000:.2f}s" for bb, ss in shapes]
        out["data"] = ("synthetic (0.1*randn waveforms; lengths uniform 2-15.6 s, bucketed and cropped like the "
                       "reference's train loader)")
    if rank == 0 and world == 1 and not args.no_cpu_baseline and batches is None and args.model == "hubert-base" \
            and args.student == "prune":
        try:
            out["cpu_baseline"] = cpu_baseline()
        except Exception as e:  # noqa: BLE001 -- baseline is informational
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
