"""The rag fusion's K = 4D projection + LN/MAF tail (gemm256 EPI 1) at the bench shape vs the
first-round stagger (option g2_desync; -1 = launcher default), interleaved repeats, HIP events."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(__file__))
os.environ.setdefault("RT_M", "527360")
import ragtail_micro as R  # noqa: E402  (operands; its timing runs at import)
from ragtail_micro import K  # noqa: E402

vals = [int(v) for v in os.environ.get("DZ", "-1,5000,10000,20000,40000").split(",")]
res = {v: [] for v in vals}
for _ in range(int(os.environ.get("REPS", 7))):
    for v in vals:
        K.set_option("g2_desync", v)
        res[v].append(R.timeit(R.wide))
K.set_option("g2_desync", -1)
print("g3 LN  " + "  ".join(f"{v}: {sorted(res[v])[len(res[v]) // 2]:.4f}" for v in vals), flush=True)
