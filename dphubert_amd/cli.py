"""Command-line entry points with the reference's flags (distill.py:147-331, final_distill.py:131-287,
prune.py:76-107, save_final_ckpt.py:8-49).  The repo-root scripts of the same names call these.

Differences from the reference, all in the plumbing around the hot path:
  * one process per GPU launched by ``torch.distributed.run`` (``--gpus N`` on a single node
    relaunches this script under it as child processes); the Lightning Trainer is replaced by
    ``dphubert_amd.trainer.Trainer`` (RCCL all-reduce, clip, fused AdamW, LR schedule);
  * checkpoints keep Lightning's layout where prune.py / save_final_ckpt.py read it:
    ``{"state_dict": {"student_model.*", "distill_linear_projs.*", ...}, "global_step", ...}``
    under ``exp_dir/ckpts/last.ckpt``; every load uses ``weights_only=True``;
  * ``--synthetic_utterances`` replaces the LibriSpeech feed by seeded 0.1*randn waveforms
    (no dataset is available offline); otherwise ``--tsv_dir`` manifests of WAV files are read
    (``dphubert_amd.data``).
"""

import argparse
import copy
import json
import logging
import os
import pathlib
import subprocess
import sys
import time

import torch
import torch.nn as nn

_LG = logging.getLogger("dphubert_amd")


# ---------------------------------------------------------------------------------------------
# argument parsers (names, defaults and choices of the reference)
# ---------------------------------------------------------------------------------------------
def _common_args(p: argparse.ArgumentParser, lr: float, warmup: int, max_updates: int):
    p.add_argument("--tsv_dir", type=pathlib.Path, default=None, help="Directory with the tsv manifests.")
    p.add_argument("--train_subset", default="train100", choices=["train100", "train960"], type=str)
    p.add_argument("--seconds_per_batch", default=87.5, type=float)
    p.add_argument("--num_workers", default=1, type=int)
    p.add_argument("--resume_checkpoint", type=pathlib.Path, default=None)
    p.add_argument("--exp_dir", default=pathlib.Path("./exp"), type=pathlib.Path)
    p.add_argument("--log_interval", default=50, type=int)
    p.add_argument("--learning_rate", default=lr, type=float)
    p.add_argument("--weight_decay", default=0.0, type=float)
    p.add_argument("--warmup_updates", default=warmup, type=int)
    p.add_argument("--max_updates", default=max_updates, type=int)
    p.add_argument("--clip_norm", default=10.0, type=float)
    p.add_argument("--num_nodes", default=1, type=int)
    p.add_argument("--gpus", default=4, type=int)
    p.add_argument("--accum_grad", default=1, type=int)
    p.add_argument("--precision", default=32, type=int,
                   help="accepted for compatibility: the HIP path always computes bf16 x bf16 -> fp32")
    p.add_argument("--teacher_ckpt", default=pathlib.Path("pretrained_ckpts/hubert-base-ls960.pth"), type=pathlib.Path)
    p.add_argument("--student_ckpt", default=pathlib.Path("pretrained_ckpts/hubert-base-ls960.pth"), type=pathlib.Path)
    p.add_argument("--distill_layers", default="0.4,8,12", type=str)
    p.add_argument("--distill_mode", type=str, default="layer2layer", choices=["layer2layer", "predlayer"])
    p.add_argument("--l2_weight", default=0.0, type=float)
    p.add_argument("--l1_weight", default=1.0, type=float)
    p.add_argument("--cos_weight", default=1.0, type=float)
    p.add_argument("--cos_type", default="raw", type=str, choices=["raw", "log_sig"])
    # build-specific
    p.add_argument("--synthetic_utterances", default=0, type=int,
                   help="train on this many seeded synthetic utterances per GPU per step instead of --tsv_dir")
    p.add_argument("--synthetic_seconds", default=10.0, type=float)
    p.add_argument("--save_interval", default=0, type=int, help="also checkpoint every N updates (0: at the end)")
    p.add_argument("--graphs", default="auto", choices=["auto", "on", "off"],
                   help="replay each optimizer step as one captured HIP graph; auto: on for fixed-shape "
                        "(--synthetic_utterances) batches, off for bucketed corpus batches (their length varies)")
    p.add_argument("--grad_comm_dtype", default="fp32", choices=["fp32", "bf16"],
                   help="payload of the data-parallel gradient all-reduce (bf16 halves the xGMI bytes)")
    p.add_argument("--reshuffle_each_epoch", action="store_true",
                   help="new batch order every epoch (the reference's DistributedBatchSampler permutes once, so by "
                        "default every epoch repeats epoch 0's order, as the reference does)")


def distill_parser():
    p = argparse.ArgumentParser(description="Joint distillation and pruning of HuBERT (MI355X)")
    _common_args(p, lr=2e-4, warmup=15000, max_updates=50000)
    p.add_argument("--pruning_units", default="conv,head,interm,attlayer,ffnlayer", type=str)
    p.add_argument("--reg_learning_rate", default=0.02, type=float)
    p.add_argument("--target_sparsity", default=0.75, type=float)
    p.add_argument("--sparsity_warmup_updates", default=5000, type=int)
    return p


def final_distill_parser():
    p = argparse.ArgumentParser(description="Final distillation of a pruned student (MI355X)")
    _common_args(p, lr=1e-4, warmup=5000, max_updates=25000)
    return p


# ---------------------------------------------------------------------------------------------
# launch helpers
# ---------------------------------------------------------------------------------------------
def _slurm_first_host(nodelist: str) -> str:
    """First host of a SLURM nodelist ("n1,n2", "gpu[03-06,09]", "a[1-2],b7")."""
    head = nodelist.split(",")[0] if "[" not in nodelist.split(",")[0] else nodelist[:nodelist.index("]") + 1]
    if "[" not in head:
        return head
    prefix, rng = head.split("[", 1)
    first = rng.rstrip("]").split(",")[0].split("-")[0]
    return prefix + first


def _slurm_env(env=None):
    """run.sh:4,48 starts one task per GPU with srun: SLURM sets SLURM_NTASKS / SLURM_PROCID / SLURM_LOCALID, not
    torch.distributed's WORLD_SIZE / RANK / LOCAL_RANK.  Returns those three (+ MASTER_ADDR / MASTER_PORT) when this
    process is one task of a multi-task srun step, else None."""
    env = os.environ if env is None else env
    if "WORLD_SIZE" in env or int(env.get("SLURM_NTASKS", "1")) <= 1 or "SLURM_PROCID" not in env:
        return None
    out = {"WORLD_SIZE": env["SLURM_NTASKS"], "RANK": env["SLURM_PROCID"],
           "LOCAL_RANK": env.get("SLURM_LOCALID", "0")}
    if "MASTER_ADDR" not in env:
        nodes = env.get("SLURM_STEP_NODELIST") or env.get("SLURM_JOB_NODELIST") or ""
        one_node = int(env.get("SLURM_NNODES", env.get("SLURM_JOB_NUM_NODES", "1"))) <= 1
        out["MASTER_ADDR"] = "127.0.0.1" if one_node or not nodes else _slurm_first_host(nodes)
    if "MASTER_PORT" not in env:
        # one port per job, shared by every task of it
        out["MASTER_PORT"] = str(20000 + int(env.get("SLURM_JOB_ID", "9531")) % 20000)
    return out


def _maybe_relaunch(args, argv):
    """Single node, --gpus N > 1, not yet under torch.distributed.run or a multi-task srun step: start it as a
    child process (never exec: nothing has touched the GPU yet, and the parent only waits)."""
    slurm = _slurm_env()
    if slurm is not None:
        os.environ.update(slurm)    # this task is one rank already (srun --ntasks-per-node, run.sh:4)
        return
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        if args.num_nodes != 1:
            raise SystemExit("multi-node: launch with torch.distributed.run on every node")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", os.environ.get("MASTER_PORT", "29531"),
               sys.argv[0]] + list(argv)
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        raise SystemExit(subprocess.call(cmd, env=env))


def _init_dist():
    slurm = _slurm_env()
    if slurm is not None:
        os.environ.update(slurm)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if not torch.cuda.is_available():
        raise SystemExit("the distill step runs on the GPU only (no CPU path)")
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, torch.device("cuda", local)


def _load(path):
    return torch.load(path, map_location="cpu", weights_only=True)


def _split_groups(distill_layers: str):
    groups = [[int(x) for x in g.split(",")] for g in distill_layers.split(".")]
    return groups, [l for g in groups for l in g]


def _projections(groups, d_s, d_t, identity: bool, mode: str = "layer2layer"):
    projs = nn.ModuleList()
    if mode == "predlayer":      # distill.py:100-107: independent Linear + GELU per distilled layer, default init
        for g in groups:
            for _ in g:
                projs.append(nn.Sequential(nn.Linear(d_s, d_t), nn.GELU()))
        return projs
    if mode != "layer2layer":
        raise ValueError(f"Invalid distill mode: {mode}")
    for g in groups:
        lin = nn.Linear(d_s, d_t)
        if identity:     # distill.py:24-26
            with torch.no_grad():
                lin.weight.copy_(torch.eye(len(lin.weight)))
                lin.bias.fill_(0)
        for _ in g:
            projs.append(lin)
    return projs


def _batches(args, rank, world, dev):
    """Yields (waveforms, lengths) on the device, forever."""
    if args.synthetic_utterances > 0:
        from .synthetic import synthetic_batch
        step = 0
        while True:
            w, ln = synthetic_batch(args.synthetic_utterances, int(args.synthetic_seconds * 16000),
                                    seed=2022 + 7919 * step + rank)
            yield w.to(dev, non_blocking=True), ln.to(dev, non_blocking=True)
            step += 1
    if args.tsv_dir is None:
        raise SystemExit("--tsv_dir is required (or --synthetic_utterances N)")
    from .data import train_loader
    epoch = 0
    while True:
        # the reference's DistributedBatchSampler permutes its batch list once (seed 0) and set_epoch does not
        # re-permute it, so every epoch repeats one order; --reshuffle_each_epoch opts into a new order per epoch
        for w, ln in train_loader(args.tsv_dir, args.train_subset, args.seconds_per_batch, args.num_workers,
                                  seed=epoch if args.reshuffle_each_epoch else 0, rank=rank, world=world):
            yield w.to(dev, non_blocking=True), ln.to(dev, non_blocking=True)
        epoch += 1
        yield None                       # epoch boundary: validation (lightning.py:302-304, 326-342)


def _validate(args, module, rank, world, dev):
    """Lightning's validation loop over the ``valid`` subset (lightning.py:302-304, 326-342): eval mode, no grad,
    the same _step; returns the mean of each logged valid_* value over this rank's share of the batches."""
    from .data import val_loader
    path = pathlib.Path(args.tsv_dir) / "valid.tsv"
    if not path.exists():
        return None
    module.eval()
    sums, n = {}, 0
    with torch.no_grad():
        for i, (w, ln) in enumerate(val_loader(args.tsv_dir, args.seconds_per_batch, args.num_workers)):
            if i % world != rank:
                continue
            module._step((w.to(dev, non_blocking=True), ln.to(dev, non_blocking=True)), i, "valid")
            for k, v in module.logged.items():
                if k.startswith("valid_"):
                    sums[k] = sums.get(k, 0.0) + float(v)
            n += 1
    module.train()
    return {k: v / max(n, 1) for k, v in sums.items()}


def _train(args, module, world, rank, dev):
    from .trainer import Trainer
    torch.manual_seed(2022)            # pl.seed_everything(2022)
    from . import ops
    ops.manual_seed(2022 + rank)
    module = module.to(dev)
    graphs = args.graphs == "on" or (args.graphs == "auto" and args.synthetic_utterances > 0)
    trainer = Trainer(module, clip_norm=args.clip_norm, accum_grad=args.accum_grad, graphs=graphs,
                      grad_dtype=torch.bfloat16 if args.grad_comm_dtype == "bf16" else torch.float32)
    ckpt_dir = args.exp_dir / "ckpts"
    if args.resume_checkpoint is not None:
        ck = _load(args.resume_checkpoint)
        module.load_state_dict(ck["state_dict"], strict=False)
        if "optimizer" in ck:
            trainer.optimizer.load_state_dict(ck["optimizer"])
        module.global_step = int(ck.get("global_step", 0))
        for _ in range(module.global_step):
            trainer.scheduler.step()
        trainer.verify_replicas()          # every rank loaded the same state (raises on all ranks otherwise)
    if rank == 0:
        ckpt_dir.mkdir(parents=True, exist_ok=True)
    log_f = open(args.exp_dir / "log.jsonl", "a") if rank == 0 else None
    feed = _batches(args, rank, world, dev)
    t0 = time.time()
    audio = 0.0
    # algorithmic work of this rank's steps (perfmodel): MFMA FLOPs and the HBM bytes of the
    # bandwidth-bound kernels -> mfma_util / hbm_gbps next to the reference's log keys (SURVEY 2 "Metrics / logging")
    from . import perfmodel as PM
    tcfg = getattr(module.teacher_model, "dph_config", None)
    scfg = getattr(module.student_model, "dph_config", None)
    n_train = sum(p.numel() for p in trainer.reducer.params)
    work_f = work_b = 0.0
    while module.global_step < args.max_updates:
        for _ in range(args.accum_grad):
            batch = next(feed)
            while batch is None:         # end of an epoch of the corpus
                val = _validate(args, module, rank, world, dev)
                if rank == 0 and val:
                    line = json.dumps(dict({"step": module.global_step}, **{k: round(v, 6) for k, v in val.items()}))
                    print(line, flush=True)
                    log_f.write(line + "\n")
                    log_f.flush()
                batch = next(feed)
            audio += batch[0].shape[0] * batch[0].shape[1] / 16000.0
            if tcfg is not None and scfg is not None:
                nb, S = batch[0].shape
                work_f += nb * PM.step_flops_per_utt(tcfg, scfg, len(module.distill_layers), S)
                work_b += nb * PM.step_hbm_bytes_per_utt(tcfg, scfg, S)
            loss = trainer.step(batch)
        work_b += PM.optimizer_hbm_bytes(n_train)
        gs = module.global_step
        if rank == 0 and (gs % args.log_interval == 0 or gs == args.max_updates):
            el = max(time.time() - t0, 1e-9)
            rec = {"step": gs, "audio_s_per_s": round(audio * world / el, 1),
                   "lr": trainer.scheduler.get_last_lr()[0]}
            if work_f > 0:
                rec["mfma_util"] = round(work_f / el / (PM.MFMA_PEAK_TFLOPS * 1e12), 4)
                rec["hbm_gbps"] = round(work_b / el / 1e9, 1)
            rec.update({k: float(v) for k, v in module.logged.items()})
            line = json.dumps(rec)
            print(line, flush=True)
            log_f.write(line + "\n")
            log_f.flush()
        if rank == 0 and args.save_interval and gs % args.save_interval == 0:
            _save(module, trainer, ckpt_dir / f"step{gs}.ckpt")
    if rank == 0:
        _save(module, trainer, ckpt_dir / "last.ckpt")
        log_f.close()
    return module


def _save(module, trainer, path):
    sd = {k: v.detach().cpu() for k, v in module.state_dict().items()}
    torch.save({"state_dict": sd, "global_step": module.global_step,
                "optimizer": trainer.optimizer.state_dict()}, path)
    _LG.info("saved %s", path)


def _init_logger(rank):
    logging.basicConfig(format="%(asctime)s - %(levelname)s - %(name)s - %(message)s", datefmt="%Y-%m-%d %H:%M:%S",
                        level=logging.INFO if rank == 0 else logging.WARN)


# ---------------------------------------------------------------------------------------------
# distill.py
# ---------------------------------------------------------------------------------------------
def distill_main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = distill_parser().parse_args(argv)
    _maybe_relaunch(args, argv)
    world, rank, dev = _init_dist()
    _init_logger(rank)
    from .lightning import DistillLoss, DistillModule
    from .trainer import units_flags
    from .wav2vec2.model import wav2vec2_model
    tck = _load(args.teacher_ckpt)
    teacher = wav2vec2_model(**tck["config"])
    res = teacher.load_state_dict(tck["state_dict"], strict=False)
    _LG.info("teacher: missing %s, unexpected %s", res.missing_keys, res.unexpected_keys)
    for p in teacher.parameters():
        p.requires_grad = False
    teacher.eval()
    sck = _load(args.student_ckpt)
    scfg = dict(sck["config"])
    scfg.update(units_flags(args.pruning_units))
    student = wav2vec2_model(**scfg)
    res = student.load_state_dict(sck["state_dict"], strict=False)
    _LG.info("student: missing %s, unexpected %s", res.missing_keys, res.unexpected_keys)
    groups, layers = _split_groups(args.distill_layers)
    projs = _projections(groups, student.encoder.feature_projection.projection.out_features,
                         teacher.encoder.feature_projection.projection.out_features, identity=True,
                         mode=args.distill_mode)
    module = DistillModule(teacher_model=teacher, student_model=student, distill_mode=args.distill_mode,
                           distill_layers=layers, distill_linear_projs=projs,
                           distill_loss=DistillLoss(args.l2_weight, args.l1_weight, args.cos_weight, args.cos_type),
                           learning_rate=args.learning_rate, weight_decay=args.weight_decay,
                           warmup_updates=args.warmup_updates, max_updates=args.max_updates, use_reg=True,
                           reg_learning_rate=args.reg_learning_rate, target_sparsity=args.target_sparsity,
                           sparsity_warmup_updates=args.sparsity_warmup_updates, tsv_dir=args.tsv_dir or ".",
                           train_subset=args.train_subset, seconds_per_batch=args.seconds_per_batch,
                           num_workers=args.num_workers)
    _train(args, module, world, rank, dev)


# ---------------------------------------------------------------------------------------------
# final_distill.py
# ---------------------------------------------------------------------------------------------
def final_distill_main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = final_distill_parser().parse_args(argv)
    _maybe_relaunch(args, argv)
    world, rank, dev = _init_dist()
    _init_logger(rank)
    from .lightning import DistillLoss, DistillModule
    from .wav2vec2.model import wav2vec2_model
    tck = _load(args.teacher_ckpt)
    teacher = wav2vec2_model(**tck["config"])
    teacher.load_state_dict(tck["state_dict"], strict=False)
    for p in teacher.parameters():
        p.requires_grad = False
    teacher.eval()
    sck = _load(args.student_ckpt)
    student = wav2vec2_model(**sck["config"])
    student.load_state_dict(sck["state_dict"], strict=False)
    groups, layers = _split_groups(args.distill_layers)
    projs = _projections(groups, student.encoder.feature_projection.projection.out_features,
                         teacher.encoder.feature_projection.projection.out_features, identity=False,
                         mode=args.distill_mode)
    projs.load_state_dict(sck["distill_linear_projs"])
    module = DistillModule(teacher_model=teacher, student_model=student, distill_mode=args.distill_mode,
                           distill_layers=layers, distill_linear_projs=projs,
                           distill_loss=DistillLoss(args.l2_weight, args.l1_weight, args.cos_weight, args.cos_type),
                           learning_rate=args.learning_rate, weight_decay=args.weight_decay,
                           warmup_updates=args.warmup_updates, max_updates=args.max_updates, use_reg=False,
                           reg_learning_rate=None, target_sparsity=None, sparsity_warmup_updates=None)
    _train(args, module, world, rank, dev)


# ---------------------------------------------------------------------------------------------
# prune.py / save_final_ckpt.py
# ---------------------------------------------------------------------------------------------
def _sub_state(state_dict, prefix):
    return {k[len(prefix):]: v for k, v in state_dict.items() if k.startswith(prefix)}


def prune_from_ckpt(distilled_ckpt, original_ckpt):
    """prune.py:13-73: rebuild the student from the distilled checkpoint, run prune(), return the
    pruned {"state_dict", "config", "distill_linear_projs"}."""
    from .wav2vec2.model import wav2vec2_model
    ck = _load(distilled_ckpt)
    ssd = _sub_state(ck["state_dict"], "student_model.")
    psd = _sub_state(ck["state_dict"], "distill_linear_projs.")
    config = dict(_load(original_ckpt)["config"])
    probe = {
        "extractor_prune_conv_channels": "feature_extractor.conv_layers.0.hard_concrete.log_alpha",
        "encoder_prune_attention_heads": "encoder.transformer.layers.0.attention.hard_concrete_for_heads.log_alpha",
        "encoder_prune_attention_layer": "encoder.transformer.layers.0.attention.hard_concrete_for_layer.log_alpha",
        "encoder_prune_feed_forward_intermediate":
            "encoder.transformer.layers.0.feed_forward.hard_concrete_for_intermediate.log_alpha",
        "encoder_prune_feed_forward_layer": "encoder.transformer.layers.0.feed_forward.hard_concrete_for_layer.log_alpha",
    }
    config.update({flag: key in ssd for flag, key in probe.items()})
    model = wav2vec2_model(**config)
    model.load_state_dict(ssd, strict=True)
    pruned_config = prune_config(model, config)
    print(json.dumps(pruned_config, indent=4))
    return {"state_dict": model.state_dict(), "config": pruned_config, "distill_linear_projs": psd}


def prune_config(model, config):
    """Call model.prune() (in place) and return the config of the pruned architecture."""
    model.eval()
    conv_config, use_attention, use_feed_forward, num_heads, remaining_heads, ff_interm = model.prune()
    pruned = copy.deepcopy(config)
    if len(num_heads) == 0:
        pruned["encoder_remaining_heads"] = remaining_heads
    else:
        pruned["encoder_num_heads"] = num_heads
    pruned.update({"extractor_conv_layer_config": conv_config, "encoder_use_attention": use_attention,
                   "encoder_use_feed_forward": use_feed_forward, "encoder_ff_interm_features": ff_interm,
                   "extractor_prune_conv_channels": False, "encoder_prune_attention_heads": False,
                   "encoder_prune_attention_layer": False, "encoder_prune_feed_forward_intermediate": False,
                   "encoder_prune_feed_forward_layer": False})
    return pruned


def load_pruned_model(ckpt_path):
    from .wav2vec2.model import wav2vec2_model
    ck = _load(ckpt_path)
    model = wav2vec2_model(**ck["config"])
    model.load_state_dict(ck["state_dict"], strict=True)
    return model


def prune_main(argv=None):
    p = argparse.ArgumentParser(description="Prune and save distilled model.")
    p.add_argument("--distilled_ckpt", type=pathlib.Path)
    p.add_argument("--original_ckpt", type=pathlib.Path)
    args = p.parse_args(argv)
    out = args.distilled_ckpt.parent / "pruned_hubert_base.pth"
    torch.save(prune_from_ckpt(args.distilled_ckpt, args.original_ckpt), out)
    load_pruned_model(out)
    print(f"Successfully saved pruned model weights and config to: {out}")


def save_final_ckpt_main(argv=None):
    p = argparse.ArgumentParser(description="Save ckpt and config after final distill.")
    p.add_argument("--config_path", type=pathlib.Path)
    p.add_argument("--ckpt_after_final_distill", type=pathlib.Path)
    args = p.parse_args(argv)
    config = _load(args.config_path)["config"]
    print(json.dumps(config, indent=4))
    ck = _load(args.ckpt_after_final_distill)
    out = args.ckpt_after_final_distill.parent / "pruned_hubert_base.pth"
    torch.save({"state_dict": _sub_state(ck["state_dict"], "student_model."), "config": config,
                "distill_linear_projs": _sub_state(ck["state_dict"], "distill_linear_projs.")}, out)
    load_pruned_model(out)
    print(f"Successfully saved pruned model weights and config to: {out}")
