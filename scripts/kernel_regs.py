#!/usr/bin/env python3
"""Per-kernel VGPR / AGPR / spill / LDS summary of one .hip file (hipcc
-Rpass-analysis=kernel-resource-usage), e.g. scripts/kernel_regs.py csrc/gemm16.hip [name-filter]."""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-I../include", "-Icsrc", "--offload-arch=gfx950",
       "-c", src, "-o", "/tmp/_regs.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z \[\]/]+?):\s+(\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = int(m.group(2))
for r in rows:
    if flt not in r["name"]:
        continue
    n = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
    n = re.sub(r"emb::\(anonymous namespace\)::", "", n)
    n = n.split("(")[0]
    print(f"{n:70s} vgpr {r.get('VGPRs', '?'):>3} agpr {r.get('AGPRs', '?'):>3} "
          f"spill {r.get('VGPRs Spill', '?'):>3} lds {r.get('LDS Size [bytes/block]', '?')}")
