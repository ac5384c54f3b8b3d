"""Per-kernel register / LDS / scratch usage of a gfx950 object built by hipcc (no GPU needed).

    python tools/kernel_resources.py dphubert_amd/csrc/build/gemm.o [name-substring]
"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = "/opt/rocm/lib/llvm/bin"


def notes(obj: str) -> str:
    with tempfile.TemporaryDirectory() as d:
        fb, co = Path(d) / "fatbin", Path(d) / "co"
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        return subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)], check=True, capture_output=True,
                              text=True).stdout


def main():
    obj = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    s = notes(obj)
    for b in re.split(r"\n\s+- \.agpr_count", s)[1:]:
        name = re.search(r"\.name:\s+(\S+)", b).group(1)
        if pat not in name:
            continue
        g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", b) or [None, "?"])[1]  # noqa: E731
        agpr = re.match(r":\s+(\d+)", b).group(1)
        print(f"vgpr {g('vgpr_count'):>4} agpr {agpr:>4} spill {g('vgpr_spill_count'):>3} "
              f"lds {g('group_segment_fixed_size'):>6} scratch {g('private_segment_fixed_size'):>4}  {name[:110]}")


if __name__ == "__main__":
    main()
