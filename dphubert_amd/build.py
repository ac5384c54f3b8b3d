"""Build the gfx950 kernel library ``dphubert_amd/libdphubert_hip.so`` in-tree.

hipcc cross-compiles for gfx950 without a GPU, so this runs in the build
container; the resulting .so travels to the GPU box with the repo snapshot.
"""

import concurrent.futures as cf
import os
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
INCLUDE = HERE.parent / "include"
LIB = HERE / "libdphubert_hip.so"
OBJ = HERE / "csrc" / "build"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", str(INCLUDE), "-Wno-unused-result"]


def _sources():
    return sorted(CSRC.glob("*.hip"))


def _compile(src: Path) -> Path:
    obj = OBJ / (src.stem + ".o")
    deps = [src] + list(CSRC.glob("*.h")) + list(INCLUDE.glob("*.h"))
    if obj.exists() and obj.stat().st_mtime >= max(d.stat().st_mtime for d in deps):
        return obj
    cmd = [HIPCC] + FLAGS + ["-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-6000:]}")
    return obj


def build(force: bool = False, jobs: int = 8) -> Path:
    OBJ.mkdir(parents=True, exist_ok=True)
    srcs = _sources()
    if force:
        for o in OBJ.glob("*.o"):
            o.unlink()
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(_compile, srcs))
    if LIB.exists() and not force and LIB.stat().st_mtime >= max(o.stat().st_mtime for o in objs):
        return LIB
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(LIB)] + [str(o) for o in objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv))
