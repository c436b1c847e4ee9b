"""Training attention kernels at the bench's train shape (B = 24 -> 48 sequences x 1030 tokens,
12 heads, dh 32): forward (+LSE) and backward launch times with and without the 0.1
attention-probability dropout (the counter-based keep mask regenerated in each kernel)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

nseq, L, H, dh = int(os.environ.get("NSEQ", 48)), 1030, 12, 32
qkv = (torch.randn(nseq * L, 3 * H * dh, device="cuda") * 0.5).to(torch.bfloat16)
dout = (torch.randn(nseq * L, H * dh, device="cuda") * 0.1).to(torch.bfloat16)
fl = 4.0 * L * L * dh * H * nseq


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return a.elapsed_time(e) / reps


for p in (0.0, 0.1):
    out, lse = K.attention_train_fwd(qkv, nseq, L, H, dh, p, 7)
    tf = timeit(lambda: K.attention_train_fwd(qkv, nseq, L, H, dh, p, 7))
    tb = timeit(lambda: K.attention_bwd(qkv, out, dout, lse, nseq, L, H, dh, p, 7))
    print(f"p={p}: fwd {tf:.4f} ms ({fl / tf / 1e9:.0f} TFLOP/s)  bwd {tb:.4f} ms ({2.5 * fl / tb / 1e9:.0f} TFLOP/s)",
          flush=True)
