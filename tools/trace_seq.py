"""Print the kernel sequence of the last forward pass in a rocprofv3 kernel trace (one line
per launch: duration, grid, VGPRs, LDS, name) and a per-kernel-class total."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
anchor = sys.argv[2] if len(sys.argv) > 2 else "af_gate"
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
s = max(0, idx[-1] - 12)
tot = defaultdict(float)
seen_ffn = 0
for r in rows[s:]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    name = r["Kernel_Name"]
    short = name.split("(")[0][-60:]
    tot[short] += d
    if "ffn_kernel" in name:
        seen_ffn += 1
    if "ffn_kernel" in name and 1 < seen_ffn < 12:
        continue
    if "attn32" in name or "wsg_kernel<384, 18" in name:
        if 1 < seen_ffn < 12:
            continue
    print(f"{d:9.1f}us {r['Grid_Size_X']:>9} {r['VGPR_Count']:>4} {r['LDS_Block_Size']:>6} {name[:70]}")
print("--- totals (us)")
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:20]:
    print(f"{v:10.1f}  {k}")
