"""Kernel resource usage (VGPRs, AGPRs, scratch, spills, occupancy) of one csrc/*.hip file,
from hipcc's -Rpass-analysis=kernel-resource-usage remarks.
usage: python tools/kres.py csrc/tail.hip [name-filter]"""
import os
import re
import subprocess
import sys

root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "rag-snvbert_amd")
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", "/tmp/kres.o",
       "-Rpass-analysis=kernel-resource-usage"] + os.environ.get("EXTRA", "").split()
out = subprocess.run(cmd, cwd=root, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark: .*?\s+([A-Za-z ]+?)(?: \[bytes/lane\])?(?: \[waves/SIMD\])?: (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
dem = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                     text=True).stdout.split("\n")
for r, d in zip(rows, dem):
    if flt in d:
        g = lambda k: r.get(k, "?")
        print(f"VGPR {g('VGPRs'):>4} AGPR {g('AGPRs'):>3} scratch {g('ScratchSize'):>4} "
              f"vspill {g('VGPRs Spill'):>3} occ {g('Occupancy')}  {d[:120]}")
