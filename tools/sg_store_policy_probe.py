"""Stream-GEMM output-store cache policy A/B (option sg_store_pol: 0 default, 1 sc0, 2 nt,
3 sc0|nt) on the QKV projection — an r6 measurement whose option was removed afterwards
(profiles/r6_sg_store_policy_probe.txt: the nt policies 2.9x / 1.4x slower, sc0 equal) and the rag fusion's cat GEMM at the bench shapes; interleaved
repeats, HIP events, and the outputs bitwise equal across policies."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

D, H, BL = 384, 1536, 256 * 1030
M = 2 * BL
g = torch.Generator(device="cpu").manual_seed(0)
rn = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).to("cuda")
wq = (rn(3 * D, D) / math.sqrt(D)).to(torch.bfloat16)
wc = (rn(H, 2 * D) / math.sqrt(2 * D)).to(torch.bfloat16)
qs, qv = K.sgemm_pack(wq), K.sgemm_vec(rn(3 * D))
cs, cv = K.sgemm_pack(wc), K.sgemm_vec(rn(H))
x = rn(M, D).to(torch.bfloat16)
r = rn(M, D).to(torch.bfloat16)
aw = torch.rand(BL, D, generator=g).to("cuda", torch.bfloat16)
cases = {"QKV": lambda: K.sgemm(x, qs, 3 * D, qv), "cat GEMM": lambda: K.sgemm_cat(x, r, aw, BL, cs, H, cv)}


def timeit(fn, pol, reps=10):
    K.set_option("sg_store_pol", pol)
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for name, fn in cases.items():
    outs = []
    for pol in range(4):
        K.set_option("sg_store_pol", pol)
        outs.append(fn().clone())
    print(name, "bitwise equal across policies:", all(torch.equal(o, outs[0]) for o in outs), flush=True)
    res = {p: [] for p in range(4)}
    for _ in range(7):
        for p in range(4):
            res[p].append(timeit(fn, p))
    for p in range(4):
        s = sorted(res[p])
        print(f"{name:9s} policy {p}: median {s[3]:.4f} ms  best {s[0]:.4f}", flush=True)
K.set_option("sg_store_pol", 0)
