"""Compact per-kernel register report of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage):
    python tools/regcheck.py csrc/winograd.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o",
                      "/tmp/regcheck.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur = None
rows = {}
for ln in out.splitlines():
    m = re.search(r"Function Name: (\S+)", ln)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", ln)
    if m and cur:
        rows[cur][m.group(1)] = int(m.group(2))
for k, v in rows.items():
    if flt in k:
        print(f"{v.get('VGPRs', 0):4d} v {v.get('AGPRs', 0):4d} a  spill {v.get('VGPRs Spill', 0):3d}/{v.get('SGPRs Spill', 0):3d}  "
              f"occ {v.get('Occupancy [waves/SIMD]', 0)}  lds {v.get('LDS Size [bytes/block]', 0):6d}  {k}")
