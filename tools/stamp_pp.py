"""Per-block timeline of the ping-pong GEMM (pp_gemm_kernel) from s_memtime stamps (diagnostic build, DPH_STAMP=1).

  python tools/stamp_pp.py build [-DDPH_PP_ABL=1|2]    # ab/stamp_pp[1|2].so (build container; 1: no main-loop
                                                       # DMAs, 2: no main-loop MFMAs -- timing ablations)
  DPH_LIB_PATH=ab/stamp_pp.so DPH_PP_FORCE=15 python tools/stamp_pp.py time M N K [resid]   (GPU box)

Stamps per block: start, prologue landed (first K-tiles in LDS), main loop done, epilogue done (after a block
barrier).  Reported in shader-clock ticks: the launch span, per-block prologue / loop / epilogue means, and the
start / end spreads over the blocks.  Only shares are meaningful (the stamps serialise the block a little); the
diagnostic build's outputs are not checked.
"""
import ctypes as C
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

if sys.argv[1] == "build":
    from dphubert_amd import build as b
    b.build()
    objs = [o for o in (REPO / "dphubert_amd" / "csrc" / "build").glob("*.o") if o.stem != "gemm"]
    (REPO / "ab").mkdir(exist_ok=True)
    extra = sys.argv[2:]          # e.g. -DDPH_PP_ABL=1 ; output ab/stamp_pp<suffix>.so
    suffix = "".join(x.split("=")[-1] for x in extra)
    obj = REPO / "ab" / f"gemm_stamp_pp{suffix}.o"
    subprocess.run([b.HIPCC] + b.FLAGS + ["-DDPH_STAMP=1"] + extra + ["-c", str(b.CSRC / "gemm.hip"), "-o", str(obj)],
                   check=True)
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o",
                    str(REPO / "ab" / f"stamp_pp{suffix}.so"), str(obj)] + [str(o) for o in objs], check=True)
    print(f"built ab/stamp_pp{suffix}.so")
else:
    import os

    import numpy as np
    import torch
    from dphubert_amd import _lib
    from dphubert_amd import kernels as K
    M, N, Kd = (int(x) for x in sys.argv[2:5])
    resid = len(sys.argv) > 5 and sys.argv[5] == "resid"
    A = (torch.rand(M, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    Cm = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    R = torch.randn(M, N, device="cuda").to(torch.bfloat16) if resid else None
    ws = torch.zeros(8 * 65536 * 8, dtype=torch.int64, device="cuda")
    args = _lib.DphGemmArgs(M, N, Kd, 1, 1, 1, 1, K.dense(A), K.dense(B), K.dense(Cm), 0, 0, 1.0, 0.0, 0, None, None,
                            None, 0, None, None, R.data_ptr() if resid else None, None, None, None, 0, 0,
                            ws.data_ptr(), ws.numel() * 8, 0, 0)
    for _ in range(5):
        _lib.call("dph_gemm", C.byref(args), _lib.stream_ptr())
    torch.cuda.synchronize()
    kind = int(os.environ.get("DPH_PP_FORCE", "15"))
    bm, bn = {12: (256, 256), 13: (128, 256), 14: (256, 128), 15: (128, 192), 16: (128, 128)}[kind]
    tiles = ((M + bm - 1) // bm) * ((N + bn - 1) // bn)
    d = ws[: 8 * tiles].view(tiles, 8).cpu().numpy().astype(np.int64)
    t0 = d[:, 0].min()
    st = d[:, :4] - t0
    pro, loop, epi = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
    print(f"{M}x{N}x{Kd}{' +resid' if resid else ''} tile {bm}x{bn}: {tiles} blocks, span {st[:, 3].max()} ticks; "
          f"per block prologue {pro.mean():.0f} loop {loop.mean():.0f} ({loop.mean() / (Kd // 64):.0f}/K-tile) "
          f"epilogue {epi.mean():.0f}; block total min/mean/max {(st[:, 3] - st[:, 0]).min()}/"
          f"{(st[:, 3] - st[:, 0]).mean():.0f}/{(st[:, 3] - st[:, 0]).max()}")
    q = lambda v: [int(np.percentile(v, p)) for p in (0, 10, 50, 90, 100)]  # noqa: E731
    print(f"  start  p0/10/50/90/100 {q(st[:, 0])}")
    print(f"  loop0  p0/10/50/90/100 {q(st[:, 1])}")
    print(f"  loopE  p0/10/50/90/100 {q(st[:, 2])}")
    print(f"  end    p0/10/50/90/100 {q(st[:, 3])}")
