"""Graph-vs-eager tracking trials in ONE process (the statistics behind tests/test_graph_gpu.py's bounds): for each
(family, accum) trial, four eager trainers and one graph trainer step the same batch; prints pass / fail of
tracks_eager_report and its whole-vector line.  usage (GPU box, repo root): python tools/graph_flake_probe.py"""
import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch
from test_graph_gpu import _batch, _module, tracks_eager_report
from dphubert_amd.trainer import Trainer
for fam, accum in [("hubert", 3), ("hubert", 3), ("hubert", 3), ("hubert", 1), ("large", 2), ("hubert", 3)]:
    batch = _batch()
    eager = [Trainer(_module(family=fam), clip_norm=10.0, accum_grad=accum) for _ in range(4)]
    gr = Trainer(_module(family=fam), clip_norm=10.0, graphs=True, graph_warmup=1, accum_grad=accum)
    le = [[] for _ in eager]; lg = []
    for _ in range(5 * accum):
        for t, l in zip(eager, le):
            l.append(t.step(batch).item())
        lg.append(gr.step(batch).item())
    torch.cuda.synchronize()
    ok, lines = tracks_eager_report(eager, gr, le, lg)
    print(fam, accum, ok, lines[-1], flush=True)
    del eager, gr
