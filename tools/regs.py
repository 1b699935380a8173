#!/usr/bin/env python3
"""Per-kernel register / spill / occupancy summary of one HIP source (hipcc -Rpass-analysis=
kernel-resource-usage), demangled names shortened: the quick check for spills after a kernel edit.
usage: tools/regs.py csrc/<file>.hip [name-substring]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-Wno-unused-function",
       "-c", src, "-o", "/tmp/_regs.o", "-Rpass-analysis=kernel-resource-usage"]
if any(k in src for k in ("wino",)):
    cmd[1:1] = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark: +([A-Za-z /\[\]]+?): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
names = subprocess.run(["c++filt"], input="\n".join(rows), capture_output=True,
                       text=True).stdout.splitlines()
for (k, v), dn in zip(rows.items(), names):
    dn = dn.replace("(anonymous namespace)::", "")
    if flt and flt not in dn:
        continue
    print(f"{dn[:90]:90s} vgpr {v.get('VGPRs', '?'):>3} agpr {v.get('AGPRs', '?'):>3} "
          f"spill {v.get('VGPRs Spill', '?')} occ {v.get('Occupancy [waves/SIMD]', '?')} lds {v.get('LDS Size [bytes/block]', '?')}")
