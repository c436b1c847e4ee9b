"""The rag fusion's fusion[3] -> LayerNorm -> MAF -> residual (fusion.py:152-162) at the bench shape
(M = 2 B L = 527 360 rows, K = 4D = 1536 -> 384): the row-panel GEMM with its LN/post epilogue
(K.linear, the r5 path) against the wide-row GEMM's EPI 1 (K.gemm256_ln) at every workgroup
height, launch times by HIP events (median of 5 x 10 launches)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

M = int(os.environ.get("RT_M", 527360))
BL = M // 2
D, Kd = 384, 1536
dev = "cuda"
g = torch.Generator(device="cpu").manual_seed(0)
a = torch.randn(M, Kd, generator=g).to(dev, torch.bfloat16)
w = (torch.randn(D, Kd, generator=g) / math.sqrt(Kd)).to(dev, torch.bfloat16)
b = torch.randn(D, generator=g).to(dev)
gm, be = torch.ones(D, device=dev), torch.zeros(D, device=dev)
base = torch.randn(M, D, generator=g).to(dev, torch.bfloat16)
af = torch.rand(BL, generator=g).to(dev)
wp = K.gemm256_pack(w)


def rows():
    return K.linear(a, w, b, ln=(gm, be), post_base=base, post_scale=0.1, post_af=af, post_af_period=BL,
                    post_maf=True)


def wide():
    return K.gemm256_ln(a, wp, b, (gm, be), base=base, post_scale=0.1, post_af=af, post_af_period=BL)


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    return sorted(ts)[2]


y0, y1 = rows(), wide()
print(f"M = {M}: max |row-panel - wide-row| {(y0.float() - y1.float()).abs().max().item():.4f}", flush=True)
fl = 2.0 * M * D * Kd
for name, fn, G in [("row-panel K.linear", rows, 0), ("gemm256_ln auto", wide, 0)] + \
        [(f"gemm256_ln G={G}", wide, G) for G in (4, 5, 6, 7, 8)]:
    K.set_option("g2_groups", G)
    t = timeit(fn)
    print(f"{name:22s} {t:.4f} ms  {fl / t / 1e9 / 2500:.3f} of 2.5 PF", flush=True)
K.set_option("g2_groups", 0)
