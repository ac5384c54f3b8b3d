"""Probe: does a whole-step HIP-graph capture work with the RCCL gradient all-reduce inside it?

Single process, world_size 1 over RCCL ("nccl" backend), GradReducer forced on so every bucket
goes through a real RCCL all-reduce (AVG) launched from the backward hooks during capture.
Compares 4 replayed optimizer steps with 4 eager steps of an identical module, bitwise (deterministic mode).
Run on the GPU box:  python tools/graph_rccl_probe.py [--comm fp32|bf16] [--accum N] [--port P]
(tests/test_graph_gpu.py::test_graph_replay_with_rccl_allreduce runs it as a subprocess)
"""
import argparse
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--comm", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--accum", type=int, default=1)
    ap.add_argument("--port", default="29533")
    args = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = args.port
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from test_graph_gpu import _batch, _module, bitwise_report
    from dphubert_amd import _lib
    from dphubert_amd.trainer import Trainer
    _lib.set_deterministic(True)
    batch = _batch()
    gd = torch.bfloat16 if args.comm == "bf16" else torch.float32
    eager = [Trainer(_module(), clip_norm=10.0, accum_grad=args.accum, grad_dtype=gd) for _ in range(2)]
    gr = Trainer(_module(), clip_norm=10.0, graphs=True, graph_warmup=1, accum_grad=args.accum, grad_dtype=gd)
    for t in eager + [gr]:
        t.reducer.force_enable()
    le = [[] for _ in eager]
    lg = []
    for _ in range(4 * args.accum):
        for t, l in zip(eager, le):
            l.append(t.step(batch).item())
        lg.append(gr.step(batch).item())
    torch.cuda.synchronize()
    print("graph captured:", gr._graph is not None, "variants:", sorted(gr._graphs))
    print("reducer buckets:", len(gr.reducer.buckets), "comm dtype:", gr.reducer.comm_dtype)
    print("eager losses  ", le)
    print("graph losses  ", lg)
    # the criteria of tests/test_graph_gpu.py::test_graph_replay_matches_eager: bitwise equal
    ok, lines = bitwise_report(eager, gr, le, lg)
    ok &= gr._graph is not None
    print("\n".join(lines))
    dist.destroy_process_group()
    print("RCCL_GRAPH_OK" if ok else "RCCL_GRAPH_FAIL")


if __name__ == "__main__":
    main()
