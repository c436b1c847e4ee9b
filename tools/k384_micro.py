"""K = 384 -> N = 384 GEMMs of training (out-projection forward and dX) at M = 49 440: the wide-row
GEMM (csrc/gemm256.hip) vs the stream GEMM (csrc/sgemm.hip) vs the row-panel GEMM."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

dev, bf = "cuda", torch.bfloat16
M = int(os.environ.get("GM_M", 49440))


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


x = torch.randn(4096, 4096, device=dev)
for _ in range(50):
    x @ x
for Kd in (384, 768):
    a = torch.randn(M, Kd, device=dev).to(bf)
    w = (torch.randn(384, Kd, device=dev) / Kd ** 0.5).to(bf)
    b = torch.randn(384, device=dev)
    wp = K.gemm256_pack(w)
    fl = 2.0 * M * 384 * Kd
    res = [("gemm256", lambda: K.gemm256(a, wp, 384, bias=b)), ("row-panel", lambda: K.linear(a, w, b))]
    if Kd == 384:
        ws = K.sgemm_pack(w)
        vec = K.sgemm_vec(b)
        res.append(("stream GEMM", lambda: K.sgemm(a, ws, 384, vec)))
        y0, y1 = K.gemm256(a, wp, 384, bias=b), K.sgemm(a, ws, 384, vec)
        print(f"K={Kd}: max|gemm256 - sgemm| {(y0.float() - y1.float()).abs().max().item():.4f}", flush=True)
    for name, fn in res + [("gemm256 again", res[0][1])]:
        ms = timeit(fn)
        print(f"  K={Kd} {name:16s} {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TFLOP/s", flush=True)
