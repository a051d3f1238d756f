"""Per-kernel register / scratch / occupancy table from hipcc's -Rpass-analysis=kernel-resource-usage remarks.
usage: python scripts/kernel_resources.py <source.hip> [filter]   (CPU: compiles for gfx950, prints one line per kernel)"""
import re
import subprocess
import sys

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-c", src, "-o",
                    "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
cur = None
rows = {}
for ln in r.stderr.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", ln)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k.split()[0]] = v
for name, d in rows.items():
    if filt in name:
        print(f"{d.get('VGPRs','?'):>4} v {d.get('AGPRs','?'):>4} a {d.get('ScratchSize','?'):>4} scr "
              f"{d.get('Occupancy','?'):>2} occ {d.get('LDS','?'):>6} lds  {name}")
