"""Bisect forward nondeterminism: snapshot every kernel call's tensor arguments across two runs."""
import sys

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from helpers import load_golden, wave_batch  # noqa: E402
from test_parity_gpu import build_module  # noqa: E402
from dphubert_amd import _lib, ops  # noqa: E402
from dphubert_amd import kernels as K  # noqa: E402

fx = load_golden(sys.argv[1] if len(sys.argv) > 1 else "g2b_all_units_padded.pt")
wave, ln = wave_batch(fx["B"], fx["S"], lengths=None if fx["lengths"] is None else fx["lengths"].tolist())
wave, ln = wave.cuda(), ln.cuda()

pending = []
log = []
orig_ptr = ops.ptr
orig_call = ops.call


def rec_ptr(t):
    if isinstance(t, torch.Tensor):
        pending.append(t)
    return orig_ptr(t)


def rec_call(name, *args):
    r = orig_call(name, *args)
    torch.cuda.synchronize()
    if name not in ("dph_cast_bf16", "dph_conv_weight_pack"):   # cached weight images: first run only
        log.append((name, [t.detach().clone() for t in pending]))
    pending.clear()
    return r


orig_lf = K.linear_fwd


def rec_lf(*a, **k):
    out = orig_lf(*a, **k)
    torch.cuda.synchronize()
    extra = [k[n] for n in ("pre_out",) if k.get(n) is not None]
    log.append(("linear_fwd", [out.detach().clone()] + [e.detach().clone() for e in extra]))
    return out


ops.ptr = rec_ptr
ops.call = rec_call
K.linear_fwd = rec_lf
dm = build_module(fx)
runs = []
for _ in range(2):
    log.clear()
    pending.clear()
    with torch.no_grad():
        dm.student_model.extract_features(wave, ln)
    runs.append(list(log))
for i, ((n1, t1), (n2, t2)) in enumerate(zip(*runs)):
    diffs = []
    for a, b in zip(t1, t2):
        if a.shape != b.shape:
            diffs.append("shape")
        elif not torch.equal(a, b):
            diffs.append(f"{(a.float() - b.float()).abs().max().item():.3g}@{tuple(a.shape)}")
    print(i, n1, "OK" if not diffs else diffs)
