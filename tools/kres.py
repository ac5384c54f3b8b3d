"""Per-kernel register / spill / occupancy summary of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage).
usage: python tools/kres.py SOURCE.hip [name-substring] [-DFOO=1 ...]"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("-D") else ""
defs = [a for a in sys.argv[2:] if a.startswith("-D")]
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I", "../../include",
                    "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"] + defs,
                   capture_output=True, text=True)
cur = None
rows = {}
for line in r.stderr.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for name, d in rows.items():
    if pat and pat not in name:
        continue
    short = re.sub(r"_ZN3dph12_GLOBAL__N_1", "", name)[:90]
    print(f"{d.get('VGPRs', 0):4d} vgpr {d.get('AGPRs', 0):3d} agpr spill {d.get('VGPRs Spill', 0):3d} "
          f"occ {d.get('Occupancy [waves/SIMD]', 0)}  {short}")
