"""Wide-row block tail at the bench shape (M = 512 x 1030): launch time vs the first-round stagger
(option tail_desync, cycles per phase step; -1 = the launcher's default 10 000), interleaved
repeats, HIP events."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
sys.path.insert(0, os.path.dirname(__file__))
from src import kernels as K  # noqa: E402
from tailw_micro_case import case  # noqa: E402

M = 512 * 1030
c = case(M, 1)
ts = K.tail_pack(c["w_o"], c["w1"], c["w2g"])
xs = c["x"].clone()


def timeit(dz, reps=10):
    K.set_option("tail_desync", dz)
    fn = lambda: K.tail_forward(c["att"], xs, ts, c["b_o"], c["g1"], c["be1"], c["vec"])
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


vals = [int(v) for v in os.environ.get("DZ", "-1,0,5000,15000,20000,30000").split(",")]
for _ in range(10):
    timeit(-1, 1)
res = {v: [] for v in vals}
for it in range(int(os.environ.get("REPS", 5))):
    for v in vals:
        res[v].append(timeit(v))
K.set_option("tail_desync", -1)
fl = 18.0 * M * 384 * 384
for v in vals:
    s = sorted(res[v])
    print(f"desync {v:6d}: median {s[len(s) // 2]:.4f} ms  best {s[0]:.4f}  ({fl / s[len(s) // 2] / 1e9 / 2500:.3f} of 2.5 PF)", flush=True)
