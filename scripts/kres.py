#!/usr/bin/env python
"""Kernel resource table (VGPRs, AGPRs, spills, occupancy) of one HIP source:
    python scripts/kres.py posecnn_amd/csrc/gemm_x6.hip [filter]
Compiles with the library's flags plus -Rpass-analysis=kernel-resource-usage."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from posecnn_amd import build  # noqa: E402

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
extra = build.FILE_FLAGS.get(os.path.basename(src), [])
cmd = ["/opt/rocm/bin/hipcc"] + build.FLAGS + extra + ["-c", src, "-o", "/tmp/kres.o",
                                                       "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if flt and flt not in r["name"]:
        continue
    dem = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    print(f"{r.get('VGPRs', '?'):>4} v {r.get('AGPRs', '?'):>3} a  spill v {r.get('VGPRs Spill', '?'):>3} "
          f"s {r.get('SGPRs Spill', '?'):>4}  occ {r.get('Occupancy [waves/SIMD]', '?'):>2}  {dem[:110]}")
