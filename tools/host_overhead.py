"""Pure host (Python + launch) cost of one distill step: the GPU is parked behind a long sleep
kernel so no host call ever waits for it.  usage: python tools/host_overhead.py [--batch 16]"""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
from dphubert_amd.synthetic import HUBERT_BASE_CONFIG, synthetic_batch  # noqa: E402
from dphubert_amd.trainer import Trainer, build_distill_module  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=16)
ap.add_argument("--profile", action="store_true")
args = ap.parse_args()
dev = torch.device("cuda", 0)
m = build_distill_module(HUBERT_BASE_CONFIG, pruning_units="conv,head,interm", distill_layers="0.4,8,12").to(dev)
m.global_step = 5000
tr = Trainer(m)
wave, ln = synthetic_batch(args.batch, 160000)
batch = (wave.to(dev), ln.to(dev))
for _ in range(3):
    tr.step(batch)
torch.cuda.synchronize()
for rep in range(3):
    torch.cuda._sleep(2_000_000_000)       # ~1 s of GPU time queued ahead
    t0 = time.perf_counter()
    tr.step(batch)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"host time per step {1e3 * (t1 - t0):.2f} ms", flush=True)
if args.profile:
    import cProfile
    import pstats
    torch.cuda._sleep(4_000_000_000)
    pr = cProfile.Profile()
    pr.enable()
    tr.step(batch)
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)
