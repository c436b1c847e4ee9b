"""The rag fusion's AF gate chain at the bench shape (M = B L = 263 680 rows, D = 384):
snvrag_af_gate + the af_adapter MLP (two launches, the [M, D] bf16 gate input written and read
back) against snvrag_mlp_afgate_forward (CrossAFInteraction in the MLP's prologue, one launch);
HIP-event launch times, median of 5 x 10."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402
from src import native as N  # noqa: E402

M = int(os.environ.get("AG_M", 263680))
D, H = 384, 1536
dev = "cuda"
g = torch.Generator(device="cpu").manual_seed(0)
rn = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).to(dev)
ag = [rn(32, 2, sc=0.8), rn(32, sc=0.1), rn(D, 32, sc=0.25), rn(D, sc=0.1), rn(D, 2, sc=0.7), rn(D, sc=0.1),
      1 + rn(D, sc=0.1), rn(D, sc=0.1)]
af, afp = torch.rand(M, generator=g).to(dev), torch.rand(M, generator=g).to(dev)
w1 = (torch.randn(H, D, generator=g) / math.sqrt(D)).to(dev, torch.bfloat16)
w2 = (torch.randn(D, H, generator=g) / math.sqrt(H)).to(dev, torch.bfloat16)
mv = torch.cat([rn(H), rn(D, sc=0.1)]).contiguous()
ws = K.mlp_pack(w1, w2)
w = N.AfGateW(*[t.contiguous().data_ptr() for t in ag], 0.1)
frags, vec = K.mlp_afgate_pack(ag, mv)


def two():
    return K.mlp(K.af_gate(af, afp, w, D, torch.bfloat16), ws, mv, epi2=0)


def one():
    return K.mlp_afgate(af, afp, frags, 0.1, ws, vec)


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


print(f"M = {M}: max |two-launch - fused| {(two().float() - one().float()).abs().max().item():.4f}", flush=True)
fl = 2.0 * M * D * H * 2
for name, fn in (("af_gate + mlp", two), ("mlp_afgate", one), ("af_gate alone", lambda: K.af_gate(af, afp, w, D, torch.bfloat16))):
    t = timeit(fn)
    print(f"{name:16s} {t:.4f} ms  ({fl / t / 1e9 / 2500:.3f} of 2.5 PF for the two GEMMs)", flush=True)
