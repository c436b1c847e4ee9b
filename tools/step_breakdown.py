"""Per-kernel breakdown of bench.py's inference step from a rocprofv3 --kernel-trace CSV:
python tools/step_breakdown.py TRACE.csv [N_STEPS]

A step starts at the kNN's lut_kernel launch that precedes each rag-gate launch (the bf16 af_gate
kernel, or since r6 the af_adapter MLP with the AF gate in its prologue; once per step); the breakdown covers the last N_STEPS complete steps (start to the next
step's start), grouped by kernel name, in ms per step, with the span (wall clock between the
step starts), the kernel-busy sum and the idle remainder."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
n_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
gate = [i for i, r in enumerate(rows)
        if "af_gate_kernelIDF16b" in r["Kernel_Name"] or "mlp_kernel<384, false, 0, true>" in r["Kernel_Name"]]
starts = []
for g in gate:
    s = max(i for i in range(g) if "lut_kernel" in rows[i]["Kernel_Name"])
    starts.append(s)
starts = starts[-(n_steps + 1):]
assert len(starts) >= 2, "need two inference steps in the trace"
n = len(starts) - 1
t = lambda i, k: int(rows[i][k])
span = (t(starts[-1], "Start_Timestamp") - t(starts[0], "Start_Timestamp")) / 1e6 / n
tot, cnt = defaultdict(float), defaultdict(int)
for i in range(starts[0], starts[-1]):
    name = rows[i]["Kernel_Name"]
    tot[name] += (t(i, "End_Timestamp") - t(i, "Start_Timestamp")) / 1e6 / n
    cnt[name] += 1
busy = sum(tot.values())
print(f"span ms/step {span:.2f}  kernel ms/step {busy:.2f}  idle {span - busy:.2f}  "
      f"launches/step {sum(cnt.values()) / n:.1f}  ({n} steps)")
for name, ms in sorted(tot.items(), key=lambda x: -x[1]):
    print(f"{ms:7.3f} ms/step {cnt[name] / n:5.1f} launches  {name[:100]}")
