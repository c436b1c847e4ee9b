"""QKV stream GEMM (8 waves) at the bench shape: launch time vs the first-round stagger (option
sg_desync; -1 = the launcher's default), interleaved repeats, HIP events."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

D, M = 384, 512 * 1030
g = torch.Generator(device="cpu").manual_seed(0)
w = (torch.randn(3 * D, D, generator=g) / math.sqrt(D)).to("cuda", torch.bfloat16)
ws, vec = K.sgemm_pack(w), K.sgemm_vec(torch.randn(3 * D, generator=g).cuda())
x = torch.randn(M, D, device="cuda").to(torch.bfloat16)


def timeit(dz, reps=10):
    K.set_option("sg_desync", dz)
    K.sgemm(x, ws, 3 * D, vec)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        K.sgemm(x, ws, 3 * D, vec)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


vals = [int(v) for v in os.environ.get("DZ", "-1,0,2500,5000,10000,15000").split(",")]
for _ in range(5):
    timeit(-1, 1)
res = {v: [] for v in vals}
for _ in range(int(os.environ.get("REPS", 7))):
    for v in vals:
        res[v].append(timeit(v))
K.set_option("sg_desync", -1)
for v in vals:
    s = sorted(res[v])
    print(f"sg_desync {v:6d}: median {s[len(s) // 2]:.4f} ms  best {s[0]:.4f}", flush=True)
