"""Probe: does a whole-step HIP-graph capture work with the RCCL gradient all-reduce inside it?

Single process, world_size 1 over RCCL ("nccl" backend), GradReducer forced on so every bucket
goes through a real RCCL all-reduce (AVG) launched from the backward hooks during capture.
Compares 4 replayed steps with 4 eager steps of an identical module.
Run on the GPU box:  python tools/graph_rccl_probe.py
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from test_graph_gpu import _batch, _module
    from dphubert_amd.trainer import Trainer
    batch = _batch()
    ea = Trainer(_module(), clip_norm=10.0)
    gr = Trainer(_module(), clip_norm=10.0, graphs=True, graph_warmup=1)
    for t in (ea, gr):
        t.reducer.enabled = True
    le, lg = [], []
    for _ in range(4):
        le.append(ea.step(batch).item())
        lg.append(gr.step(batch).item())
    torch.cuda.synchronize()
    print("graph captured:", gr._graph is not None)
    print("eager losses ", le)
    print("graph losses ", lg)
    pa = dict(ea.module.named_parameters())
    worst = 0.0
    for n, p in gr.module.named_parameters():
        if p.requires_grad and not n.endswith("k_proj.bias"):   # zero-gradient param (see tests)
            d = ((p.detach() - pa[n].detach()).norm() / pa[n].detach().norm().clamp_min(1e-30)).item()
            worst = max(worst, d)
    print("worst param rel diff", worst)
    dist.destroy_process_group()
    ok = gr._graph is not None and worst < 1e-3 and all(abs(a - b) < 1e-4 for a, b in zip(le, lg))
    print("RCCL_GRAPH_OK" if ok else "RCCL_GRAPH_FAIL")


if __name__ == "__main__":
    main()
