"""Top kernels of a rocprofv3 --stats run: python tools/prof_top.py DIR [N] — reads the
*kernel_stats.csv under DIR and prints the N kernels with the most total time (ms), their call
count and average, and the sum over all kernels."""
import csv
import glob
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = []
for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((float(r["TotalDurationNs"]) / 1e6, int(r["Calls"]), r["Name"]))
rows.sort(reverse=True)
tot = sum(r[0] for r in rows)
print(f"all kernels: {tot:.2f} ms over {sum(r[1] for r in rows)} dispatches")
for ms, calls, name in rows[:n]:
    print(f"{ms:9.2f} ms {100 * ms / tot:5.1f}% {calls:6d} x {ms / calls * 1e3:8.1f} us  {name[:110]}")
