"""Run the same distill step twice (identical inputs / noise) and report gradient differences.

Atomic fp32 accumulation order makes some reductions run-to-run nondeterministic at the ~1e-7
relative level; anything much larger points at a race.
usage: python tools/determinism.py [fixture]
"""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from helpers import load_golden, rel_l2  # noqa: E402
from test_parity_gpu import run_gpu_step  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "g2b_all_units_padded.pt"
fx = load_golden(name)
runs = []
for _ in range(3):
    dm, loss, hs = run_gpu_step(fx)
    runs.append(({n: p.grad.detach().clone() for n, p in dm.named_parameters() if p.grad is not None},
                 [h.detach().clone() for h in hs], loss.item()))
print("loss", [r[2] for r in runs])
for i, (a, b) in enumerate(zip(runs[0][1], runs[1][1])):
    print(f"hidden {i} max|diff| {(a.float() - b.float()).abs().max().item():.3g}")
rows = []
for n in runs[0][0]:
    e1 = rel_l2(runs[1][0][n].cpu(), runs[0][0][n].cpu())
    e2 = rel_l2(runs[2][0][n].cpu(), runs[0][0][n].cpu())
    rows.append((max(e1, e2), n))
rows.sort(reverse=True)
for e, n in rows[:25]:
    print(f"{e:.3e}  {n}")
