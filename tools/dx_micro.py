"""Row-panel GEMM at the training dX / FFN-down shapes (M = 2 * 24 * 1030 rows, N = 384 outputs,
K = 1536 / 1152): tile width (snvrag option gemm_nw: 6 = whole 384-column rows, one round and a
half of 387 workgroups; 2 / 1 = 128 / 64 columns, more and smaller workgroups) and torch.matmul
(hipBLASLt) on the same operands.  Operands rotated over 3 copies (every launch reads HBM)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

M = int(os.environ.get("M", 2 * 24 * 1030))
N = 384
for Kd in (1536, 1152):
    xs = [torch.randn(M, Kd, device="cuda").bfloat16() for _ in range(3)]
    w = (torch.randn(N, Kd, device="cuda") / Kd ** 0.5).bfloat16()
    ref = (xs[0].float() @ w.float().t())
    for nw in (0, 2, 1, -1):
        def run(i):
            return xs[i % 3] @ w.t() if nw < 0 else K.linear(xs[i % 3], w)
        if nw >= 0:
            K.set_option("gemm_nw", nw)
        y = run(0)
        err = (y.float() - ref).abs().max().item()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(30):
            run(i)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 30
        print(f"K={Kd} {'torch' if nw < 0 else f'nw={nw}'}: {ms * 1e3:.1f} us "
              f"{2 * M * N * Kd / ms / 1e9:.0f} TF/s  max|err| {err:.3f}", flush=True)
    K.set_option("gemm_nw", 0)
