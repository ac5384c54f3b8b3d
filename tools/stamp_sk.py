"""Per-block timeline of the stream-K GEMM (sk_gemm_kernel) from s_memtime stamps (diagnostic build, DPH_STAMP=1).

  python tools/stamp_sk.py build                   # ab/stamp_sk.so (build container)
  DPH_LIB_PATH=ab/stamp_sk.so python tools/stamp_sk.py time M N K [gelu]   (GPU box)

Per logical block: start, then per segment (tail piece / whole tile / head piece) the main-loop entry (after a head
piece's wait and partial load), loop done and segment done.  Reported in shader-clock ticks relative to the earliest
start: loop ticks per K-tile, head-piece waits, epilogue / hand-off costs and the end spread.
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
    objs = [o for o in (REPO / "dphubert_amd" / "csrc" / "build").glob("*.o") if o.stem != "gemm_sk"]
    (REPO / "ab").mkdir(exist_ok=True)
    obj = REPO / "ab" / "gemm_sk_stamp.o"
    subprocess.run([b.HIPCC] + b.FLAGS + ["-DDPH_STAMP=1", "-c", str(b.CSRC / "gemm_sk.hip"), "-o", str(obj)],
                   check=True)
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", str(REPO / "ab" / "stamp_sk.so"),
                    str(obj)] + [str(o) for o in objs], check=True)
    print("built ab/stamp_sk.so")
else:
    import os

    import numpy as np
    import torch
    from dphubert_amd import _lib
    from dphubert_amd import kernels as K
    os.environ.setdefault("DPH_GEMM_SK", "1")
    M, N, Kd = (int(x) for x in sys.argv[2:5])
    act = K.ACT_GELU if len(sys.argv) > 5 and sys.argv[5] == "gelu" else K.ACT_NONE
    A = (torch.rand(M, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    Cm = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ws = torch.zeros(256 * 16, dtype=torch.int64, device="cuda")
    spans = []
    for rep in range(6):
        args = _lib.DphGemmArgs(M, N, Kd, 1, 1, 1, 1, K.dense(A), K.dense(B), K.dense(Cm), K.OUT_BF16, act, 1.0)
        args.workspace, args.workspace_bytes = ws.data_ptr(), ws.numel() * 8
        keep = K._sk_scratch(args, "cuda")
        assert keep is not None, "shape not routed to stream-K"
        nblk = int(keep[1].numel()) - 1
        _lib.call("dph_gemm", C.byref(args), _lib.stream_ptr())
        torch.cuda.synchronize()
        assert int(keep[1].view(torch.int32)[nblk]) == 0, "lost-producer flag set"
    nk = Kd // 64
    d = ws[: nblk * 16].view(nblk, 16).cpu().numpy().astype(np.int64)
    t0 = d[:, 0].min()
    st = np.where(d > 0, d - t0, -1)
    print(f"{M}x{N}x{Kd} act {act}: {nblk} blocks, nk {nk}, span {st.max()} ticks")
    segs = []
    for blk in range(nblk):
        s = 0
        while 3 * s + 3 < 16 and st[blk, 3 * s + 3] >= 0 and (s == 0 or st[blk, 3 * s + 1] >= st[blk, 3 * s]):
            segs.append((blk, s, st[blk, 3 * s + 1] - (st[blk, 0] if s == 0 else st[blk, 3 * s]),
                         st[blk, 3 * s + 2] - st[blk, 3 * s + 1], st[blk, 3 * s + 3] - st[blk, 3 * s + 2]))
            s += 1
    a = np.array(segs)
    print(f"  segments {len(a)}; entry gap (wait / partial load) mean {a[:, 2].mean():.0f} max {a[:, 2].max()}; "
          f"loop mean {a[:, 3].mean():.0f}; epilogue / hand-off mean {a[:, 4].mean():.0f} max {a[:, 4].max()}")
    q = lambda v: [int(np.percentile(v, p)) for p in (0, 10, 50, 90, 100)]  # noqa: E731
    ends = np.array([st[blk][st[blk] >= 0].max() for blk in range(nblk)])
    print(f"  start p0/10/50/90/100 {q(st[:, 0])}")
    print(f"  end   p0/10/50/90/100 {q(ends)}")
    for blk in (0, 1, nblk // 2, nblk - 1):
        print(f"  block {blk}: " + " ".join(str(x) for x in st[blk] if x >= 0))
