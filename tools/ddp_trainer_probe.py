"""Two data-parallel ranks through the FULL Trainer on one GPU (gloo backend: SUM + divide, the CPU-side twin of
the RCCL AVG path), each rank with its own bucketed batch length (audio_dataset.py:145-217: the bucketed sampler
hands every rank its own padded length), eager steps.  Checks, on every rank:
  * the all-reduced gradient buckets equal the average of the two ranks' LOCAL gradients (each rank's gradient of
    its own batch on a fresh module copy, plain autograd with the HIP kernels, no reducer), rel-L2 <= 1e-4 per
    parameter (the Trainer's grouped / deferred weight-gradient launches sum in another fp32 order);
  * both ranks launched their bucket collectives in the same order (distill.py:41 DDP: buckets paired by order);
  * after each optimizer step every parameter is bitwise identical across the ranks.
With --accum A each optimizer step is A micro-steps of the same batch (the backward is seeded with 1 / A, so the
accumulated, reduced gradient is again the mean of the local gradients; the collectives run once, on the last);
--comm bf16 sends bf16 bucket copies (tolerance 2^-8 relative).
Prints DDP_TRAINER_OK on success.  usage: python tools/ddp_trainer_probe.py --port P [--steps 2] [--accum A] [--comm bf16]
"""
import argparse
import os
import sys
from pathlib import Path

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

LENGTHS = {0: (24000, [24000, 19000]), 1: (32000, [32000, 26500])}   # rank -> (padded S, per-utterance lengths)


def _batch(rank):
    from helpers import wave_batch
    S, ln = LENGTHS[rank]
    wave, lens = wave_batch(2, S, seed=100 + rank, lengths=ln)
    return wave.cuda(), lens.cuda()


def _worker(rank, world, port, steps, accum, comm, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from test_graph_gpu import _module
        from dphubert_amd.trainer import Trainer
        batch = _batch(rank)
        # local gradient of this rank's batch (fresh copy, no reducer)
        ref = _module()
        loss = ref._step(batch, 0, "train")
        loss.backward()
        torch.cuda.synchronize()
        local = {n: p.grad.detach().clone() for n, p in ref.named_parameters() if p.grad is not None}
        del ref
        names = sorted(local)
        expect = {}
        for n in names:
            t = local[n].cpu()
            dist.all_reduce(t)
            expect[n] = t / world
        dm = _module()
        # (no clip: the buckets keep the reduced gradients after AdamW; 8 MB buckets: several collectives per step)
        tr = Trainer(dm, clip_norm=1e9, bucket_mb=8.0, accum_grad=accum,
                     grad_dtype=torch.bfloat16 if comm == "bf16" else torch.float32)
        # (accumulation seeds each micro-step's backward with 1 / A: the bf16 activation gradients then round
        # differently from the local reference's seed-1 backward -- 0.02-0.3 % per tensor -- whereas a missing or
        # doubled micro-step is a 33-200 % error)
        tol = 1e-2 if (comm == "bf16" or accum > 1) else 1e-4
        order = []
        orig = tr.reducer._launch

        def spy(bi):
            order.append(bi)
            return orig(bi)

        tr.reducer._launch = spy
        named = dict(dm.named_parameters())
        bad = []
        for step in range(steps):
            order.clear()
            for _ in range(accum):
                tr.step(batch)
            torch.cuda.synchronize()
            orders = [None] * world
            dist.all_gather_object(orders, list(order))
            if orders[0] != orders[1]:
                bad.append(f"step {step}: bucket launch order differs {orders}")
            if step == 0:
                for n in names:
                    p = named[n]
                    got = tr.reducer.views[id(p)].detach().cpu()
                    want = expect[n].double()
                    e = ((got.double() - want).norm() / want.norm().clamp_min(1e-30)).item()
                    if not (e <= tol or expect[n].abs().max().item() == 0):
                        bad.append(f"{n}: reduced grad vs mean of local grads rel-L2 {e:.3g}")
            for n, p in named.items():
                t = p.detach().cpu().clone()
                o = t.clone()
                dist.broadcast(o, src=0)
                if not torch.equal(t, o):
                    bad.append(f"step {step}: {n} differs across ranks")
        q.put((rank, len(names), len(order), bad))
    finally:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--accum", type=int, default=1)
    ap.add_argument("--comm", default="fp32")
    a = ap.parse_args()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, a.port, a.steps, a.accum, a.comm, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    ok = all(p.exitcode == 0 for p in procs)
    for rank, nparams, nbuckets, bad in sorted(res):
        print(f"rank {rank}: {nparams} gradients checked, {nbuckets} bucket collectives per step, "
              f"{len(bad)} problems")
        for b in bad[:20]:
            print("  ", b)
        ok = ok and not bad
    if ok:
        print("DDP_TRAINER_OK")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
