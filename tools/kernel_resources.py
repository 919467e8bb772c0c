#!/usr/bin/env python3
"""Per-kernel register / LDS / occupancy table of one libbmfr source, from the
compiler's kernel-resource-usage remarks (no GPU needed).

  python tools/kernel_resources.py [bmfr_fused_cols.hip] [extra hipcc flags...]
"""
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bmfr_amd import _build as b  # noqa: E402

src = sys.argv[1] if len(sys.argv) > 1 else "bmfr_fused_cols.hip"
cmd = [b.HIPCC, *b.FLAGS, *sys.argv[2:], "-Rpass-analysis=kernel-resource-usage", "-c",
       os.path.join(b.CSRC, src), "-o", "/tmp/kernel_resources.o"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass-analysis", line)
    if not m:
        continue
    txt = m.group(1).strip()
    if txt.startswith("Function Name:"):
        cur = {"name": txt.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in txt:
        k, v = txt.split(":", 1)
        cur[k.strip()] = v.strip()
keys = ["VGPRs", "AGPRs", "VGPRs Spill", "SGPRs Spill", "LDS Size [bytes/block]", "Occupancy [waves/SIMD]"]
print(f"{'kernel':70s} " + " ".join(f"{k.split(' ')[0][:8]:>8s}" for k in keys))
for r in rows:
    name = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
    print(f"{name[:70]:70s} " + " ".join(f"{r.get(k, '-'):>8s}" for k in keys))
