"""Graph replay vs eager parameter drift after 5 steps (test_graph_gpu's setup), all params listed
worst-first with the eager-vs-eager baseline.  Run on the GPU box."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from helpers import rel_l2  # noqa: E402
from test_graph_gpu import _batch, _module  # noqa: E402


def main():
    from dphubert_amd.trainer import Trainer
    batch = _batch()
    ea = Trainer(_module(), clip_norm=10.0)
    eb = Trainer(_module(), clip_norm=10.0)
    gr = Trainer(_module(), clip_norm=10.0, graphs=True, graph_warmup=1)
    for _ in range(int(os.environ.get("NSTEPS", "5"))):
        print("loss", ea.step(batch).item(), eb.step(batch).item(), gr.step(batch).item())
    torch.cuda.synchronize()
    pa, pb = dict(ea.module.named_parameters()), dict(eb.module.named_parameters())
    rows = []
    for n, p in gr.module.named_parameters():
        if p.requires_grad:
            rows.append((rel_l2(p.detach().cpu(), pa[n].detach().cpu()), rel_l2(pb[n].detach().cpu(),
                                                                               pa[n].detach().cpu()), n))
    for e, b, n in sorted(rows, reverse=True)[:15]:
        print(f"{e:.3e} base {b:.3e} {n}")


if __name__ == "__main__":
    main()
