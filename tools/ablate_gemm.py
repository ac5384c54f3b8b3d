"""Build timing-ablation variants of the ring GEMM into ab/abl<N>.so (build container), or time one
shape with whatever library DPH_LIB_PATH selects (GPU box).

  python tools/ablate_gemm.py build            # ab/abl0.so .. ab/abl6.so
  DPH_LIB_PATH=ab/abl1.so DPH_GEMM_PATH=big python tools/ablate_gemm.py time M N K
Variants: 0 production, 1 no DMA in the loop, 2 no MFMA, 3 no barrier, 4 no fragment reads
5 no epilogue, 6 no k-loop
(outputs are wrong for 1-6; only their timing is meaningful).
"""
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
    # abl0..abl6: DPH_ABLATE variants; extra args "stgN" build ab/stgN.so with DPH_STAGGER=N
    variants = sys.argv[2:] or [str(n) for n in range(7)]
    for n in variants:
        flag = f"-DDPH_STAGGER={n[3:]}" if n.startswith("stg") else f"-DDPH_ABLATE={n}"
        name = n if n.startswith("stg") else f"abl{n}"
        obj = REPO / "ab" / f"gemm_{name}.o"
        subprocess.run([b.HIPCC] + b.FLAGS + [flag, "-c", str(b.CSRC / "gemm.hip"), "-o", str(obj)], check=True)
        subprocess.run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", str(REPO / "ab" / f"{name}.so"),
                        str(obj)] + [str(o) for o in objs], check=True)
        print("built", name)
else:
    import torch
    from dphubert_amd import kernels as K
    M, N, Kd = (int(x) for x in sys.argv[2:5])
    ak = sys.argv[5] != "0" if len(sys.argv) > 5 else True       # operand layouts: 1 k-contiguous, 0 mn
    bk = sys.argv[6] != "0" if len(sys.argv) > 6 else True
    splits = int(sys.argv[7]) if len(sys.argv) > 7 else 1
    A = (torch.rand(M, Kd, device="cuda") * 2 - 1).to(torch.bfloat16) if ak else \
        (torch.rand(Kd, M, device="cuda") * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, Kd, device="cuda") * 2 - 1).to(torch.bfloat16) if bk else \
        (torch.rand(Kd, N, device="cuda") * 2 - 1).to(torch.bfloat16)
    C = torch.empty(M, N, device="cuda", dtype=torch.float32 if splits > 1 else torch.bfloat16)
    f = lambda: K.gemm(K.dense(A), K.dense(B), K.dense(C), M, N, Kd, a_kcontig=ak, b_kcontig=bk,  # noqa: E731
                       c_dtype=K.OUT_F32 if splits > 1 else K.OUT_BF16, splits=splits)
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(10):
        f()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"{os.environ.get('DPH_LIB_PATH', 'prod')} {M}x{N}x{Kd}: {ms * 1e3:.1f} us  {2 * M * N * Kd / ms / 1e9:.0f} TF/s")
