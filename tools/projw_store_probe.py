"""Does the wide-row projection (csrc/tailw.hip projw_kernel) wait on its output stores?  QKV shape
(M = 512 x 1030, D = 384, N = 3D): proj_wide 1 (normal) vs 2 (no output stores, diagnostic) vs the
8-wave stream GEMM; HIP-event launch times, median of 5 x 10.  (r6 measurement; the no-store
instantiation behind proj_wide 2 was removed afterwards, so today both projw rows run the same kernel:
profiles/r6_projw_store_probe*.txt hold the results.)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

D, dev, bf = 384, "cuda", torch.bfloat16
g = torch.Generator(device="cpu").manual_seed(0)
w = (torch.randn(3 * D, D, generator=g) / D ** 0.5).to(dev, bf)
b = (0.1 * torch.randn(3 * D, generator=g)).to(dev)
ws, sgw, sgv = K.proj_pack(w), K.sgemm_pack(w), K.sgemm_vec(b)
M = 512 * 1030
x = torch.randn(M, D, device=dev).to(bf)
out = torch.empty(M, 3 * D, device=dev, dtype=bf)


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(e) / reps)
    return sorted(ts)[2]


def pw(v):
    def fn():
        K.set_option("proj_wide", v)
        K.proj_forward(x, ws, b, 3, out=out)
    return fn


fl = 2.0 * M * D * 3 * D
for name, fn in (("projw", pw(1)), ("projw no stores", pw(2)), ("sgemm 8 waves", lambda: K.sgemm(x, sgw, 3 * D, sgv)),
                 ("projw again", pw(1))):
    t = timeit(fn)
    print(f"{name:18s} {t:.4f} ms  {fl / t / 1e9 / 2500:.3f} of 2.5 PF", flush=True)
K.set_option("proj_wide", 1)
