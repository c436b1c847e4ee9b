"""Per-dispatch averages of rocprofv3 --pmc counters for the kernels whose name contains a
filter, over every pass directory given: python tools/pmc_kernel.py FILTER DIR [DIR ...]
(counter values are summed over a dispatch's rows first: rocprofv3 writes one row per XCD /
instance for some counters)."""
import csv
import glob
import os
import sys
from collections import defaultdict

flt, dirs = sys.argv[1], sys.argv[2:]
per = defaultdict(lambda: defaultdict(float))        # (kernel, dispatch) -> counter -> value
for d in dirs:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if flt not in r["Kernel_Name"]:
                continue
            per[(r["Kernel_Name"][:60], r.get("Dispatch_Id", ""), d)][r["Counter_Name"]] += float(r["Counter_Value"])
agg = defaultdict(lambda: defaultdict(list))
for (k, _, _), cs in per.items():
    for c, v in cs.items():
        agg[k][c].append(v)
for k, cs in agg.items():
    print(k)
    for c in sorted(cs):
        vs = cs[c]
        print(f"  {c:28s} {sum(vs) / len(vs):16.4g}  (n={len(vs)})")
