"""Per-block timeline of the ring GEMM from s_memtime stamps (diagnostic build, DPH_STAMP=1).

  python tools/stamp_gemm.py build                    # ab/stamp.so (build container)
  DPH_LIB_PATH=ab/stamp.so DPH_GEMM_PATH=mid python tools/stamp_gemm.py time M N K   (GPU box)
Stamps: block start, prologue landed, main loop done, epilogue done (+ HW_ID / XCC_ID).  Only the
shares are meaningful (stamps serialize), the outputs are not written.
"""
import ctypes as C
import os
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
    extra = sys.argv[2:]          # e.g. -DDPH_EPI_VARIANT=1 ; output ab/stamp<suffix>.so
    suffix = "".join(x.split("=")[-1] for x in extra)
    obj = REPO / "ab" / f"gemm_stamp{suffix}.o"
    subprocess.run([b.HIPCC] + b.FLAGS + ["-DDPH_STAMP=1"] + extra + ["-c", str(b.CSRC / "gemm.hip"), "-o", str(obj)],
                   check=True)
    subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o",
                    str(REPO / "ab" / f"stamp{suffix}.so"), str(obj)] + [str(o) for o in objs], check=True)
    print(f"built ab/stamp{suffix}.so")
else:
    import numpy as np
    import torch
    from dphubert_amd import _lib
    from dphubert_amd import kernels as K
    M, N, Kd = (int(x) for x in sys.argv[2:5])
    A = (torch.rand(M, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, Kd, device="cuda") * 2 - 1).to(torch.bfloat16)
    Cm = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ws = torch.zeros(8 * 65536 * 8, dtype=torch.int64, device="cuda")
    args = _lib.DphGemmArgs(M, N, Kd, 1, 1, 1, 1, K.dense(A), K.dense(B), K.dense(Cm), 0, 0, 1.0, 0.0, 0, None, None,
                            None, 0, None, None, None, None, None, None, 0, 0, ws.data_ptr(), ws.numel() * 8, 0, 0)
    for _ in range(5):
        _lib.call("dph_gemm", C.byref(args), _lib.stream_ptr())
    torch.cuda.synchronize()
    bm, bn = {"big": (256, 256), "wide": (256, 128), "flat": (128, 256), "tall": (256, 64),
              "half": (128, 64)}.get(os.environ.get("DPH_GEMM_PATH", ""), (128, 128))
    tiles = ((M + bm - 1) // bm) * ((N + bn - 1) // bn)
    d = ws[: 16 * tiles].view(tiles, 16).cpu().numpy().astype(np.int64)
    t0 = d[:, 0].min()
    st = d[:, :4] - t0
    pro = st[:, 1] - st[:, 0]
    loop = st[:, 2] - st[:, 1]
    epi = st[:, 3] - st[:, 2]
    tot = st[:, 3].max()
    sa, sb, sc = d[:, 6] - d[:, 2], d[:, 7] - d[:, 6], d[:, 8] - d[:, 7]
    print(f"  epilogue split: loop->barrier {sa.mean():.0f}, LDS staging+barrier {sb.mean():.0f}, "
          f"tile_epi {sc.mean():.0f}, rest (final barrier) {(d[:, 3] - d[:, 8]).mean():.0f}")
    print(f"{M}x{N}x{Kd} blocks {tiles}: span {tot} ticks; per block mean prologue {pro.mean():.0f} "
          f"loop {loop.mean():.0f} epilogue {epi.mean():.0f} (min/max total {(st[:,3]-st[:,0]).min()}/"
          f"{(st[:,3]-st[:,0]).max()})")
    # concurrency: blocks resident per CU (xcc, se, sh, cu)
    hw = d[:, 4]
    cu = (d[:, 5] & 0xF) * 1000 + ((hw >> 13) & 0x7) * 100 + ((hw >> 12) & 1) * 20 + ((hw >> 8) & 0xF)
    u, cnt = np.unique(cu, return_counts=True)
    print(f"distinct CUs {len(u)}; blocks per CU min {cnt.min()} max {cnt.max()} mean {cnt.mean():.2f}")
    starts = np.sort(st[:, 0])
    print("start-time deciles:", [int(starts[int(q * (len(starts) - 1))]) for q in np.linspace(0, 1, 11)])
    ends = np.sort(st[:, 3])
    print("end-time deciles:  ", [int(ends[int(q * (len(ends) - 1))]) for q in np.linspace(0, 1, 11)])
    np.save(REPO / "gpurun_out" / f"stamp_{M}_{N}_{Kd}_{os.environ.get('DPH_GEMM_PATH','auto')}.npy", d)
