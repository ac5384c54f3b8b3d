"""Print per-tensor relative errors of the HardConcrete logit gradients vs a golden fixture.

usage: python tools/grad_diag.py [fixture ...] [--repeat N]
"""
import argparse
import sys

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from helpers import load_golden, rel_l2  # noqa: E402
from test_parity_gpu import run_gpu_step  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("fixtures", nargs="*", default=["g2_smoke_step.pt", "g2b_all_units_padded.pt"])
ap.add_argument("--repeat", type=int, default=1)
args = ap.parse_args()
for name in args.fixtures:
    fx = load_golden(name)
    for rep in range(args.repeat):
        dm, loss, _ = run_gpu_step(fx)
        sd = dict(dm.student_model.named_parameters())
        print(name, rep, "loss", loss.item(), fx["loss"].item())
        for n, g in fx["log_alpha_grads"].items():
            print(f"  {n:70s} {rel_l2(sd[n].grad.cpu(), g):.4f}  |g|={g.norm():.4g}")
