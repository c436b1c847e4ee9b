"""Stream GEMM (csrc/sgemm.hip) vs torch.matmul (hipBLASLt) at the training shapes with K = 384
(M = 2 * 24 * 1030 rows; q/k/v N = 1152, w_1 N = 1536, out-projection / dX N = 384)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

M = int(os.environ.get("M", 2 * 24 * 1030))
Kd = 384
for N in (1152, 1536, 384):
    xs = [torch.randn(M, Kd, device="cuda").bfloat16() for _ in range(3)]
    w = (torch.randn(N, Kd, device="cuda") / Kd ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda") * 0.1
    ws, vec = K.sgemm_pack(w), b.float().contiguous()
    for name, fn in (("sgemm", lambda i: K.sgemm(xs[i % 3], ws, N, vec)),
                     ("torch", lambda i: torch.addmm(b.bfloat16(), xs[i % 3], w.t()))):
        fn(0)
        torch.cuda.synchronize()
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(30):
            fn(i)
        e.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(e) / 30
        print(f"N={N} {name}: {ms * 1e3:.1f} us {2 * M * N * Kd / ms / 1e9:.0f} TF/s", flush=True)
