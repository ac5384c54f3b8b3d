"""What the teacher forward costs inside the replayed step: the default bench step (HuBERT-Base, B = 16 x 10 s, HIP
graph) timed as is, then with the teacher's extract_features replaced by its cached outputs (a DIAGNOSTIC only: the
step then skips work), same process.  The difference is the part of the step the concurrent teacher stream does
not hide -- the most that moving the teacher beside other phases of the step could recover.

    python tools/teacher_cost.py [steps]
"""
import sys
import time

import torch

sys.path.insert(0, ".")


def run(steps, cached, overlap=False):
    from dphubert_amd import ops
    from dphubert_amd.synthetic import HUBERT_BASE_CONFIG, synthetic_batch
    from dphubert_amd.trainer import Trainer, build_distill_module
    ops.manual_seed(2022)
    dm = build_distill_module(HUBERT_BASE_CONFIG).cuda()
    dm.global_step = 5000
    w, l = synthetic_batch(16, 160000, seed=2022)
    batch = (w.cuda(), l.cuda())
    if cached:
        with torch.no_grad():
            out = dm.teacher_model.extract_features(*batch)
        real = dm.teacher_model.extract_features
        if overlap:
            # the schedule of a teacher prefetched one step ahead: the real teacher forward forked onto its own
            # stream (outputs discarded), joined only at the end of the step, beside the student loss / backward
            side = torch.cuda.Stream()
            dm.teacher_stream = None

            def tf(*a, **k):
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side), torch.no_grad(), ops.private_zero_arena(dm._teacher_arena):
                    real(*a, **k)
                return out
            dm.teacher_model.extract_features = tf
        else:
            dm.teacher_model.extract_features = lambda *a, **k: out
    tr = Trainer(dm, clip_norm=10.0, graphs=True, graph_warmup=2)
    if cached and overlap:
        orig = tr._gpu_step

        def gs(*a, **k):
            r = orig(*a, **k)
            torch.cuda.current_stream().wait_stream(side)
            return r
        tr._gpu_step = gs
    for _ in range(5):
        tr.step(batch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step(batch)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    for rep in range(2):
        a = run(n, False)
        b = run(n, True)
        c = run(n, True, overlap=True)
        print(f"rep {rep}: step {a:.3f} ms, teacher cached {b:.3f} ms, teacher cost in the step {a - b:.3f} ms; "
              f"teacher beside the loss / backward {c:.3f} ms", flush=True)
