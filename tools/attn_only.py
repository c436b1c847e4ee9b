"""Run only the bf16 dh=32 attention kernel at the bench shape (512 sequences x 1030 tokens,
12 heads) — for rocprofv3 PMC passes and timing."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

nseq, L, H, dh = int(os.environ.get("NSEQ", 512)), 1030, 12, 32
qkv = (torch.randn(nseq * L, 3 * H * dh, device="cuda") * float(os.environ.get("QKV_STD", 0.4))).to(torch.bfloat16)
# PRESCALED=1 (default): Q carries log2(e)/sqrt(dh) as in the engine (the QKV epilogue's q_scale),
# so the bench's attn32_dma<true> runs; PRESCALED=0: the unscaled-Q kernel
pre = os.environ.get("PRESCALED", "1") == "1"
scale = 1.0 / math.log2(math.e) if pre else 1.0 / math.sqrt(dh)
if pre:
    qkv[:, :H * dh] = (qkv[:, :H * dh].float() * (math.log2(math.e) / math.sqrt(dh))).to(torch.bfloat16)
base = None
# ATTN_VARIANTS="0,1,2,3": the inference kernel's A/B variants (snvrag option attn_variant), each
# timed and checked bit for bit against variant 0; rounds alternate to spread DVFS drift
variants = [int(v) for v in os.environ.get("ATTN_VARIANTS", "0").split(",")]
reps = int(os.environ.get("REPS", 3))
res = {v: [] for v in variants}
for rnd in range(int(os.environ.get("ROUNDS", 1))):
    for v in variants:
        K.set_option("attn_variant", v)
        out = None
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for i in range(reps):
            if i == 1:
                a.record()
            out = K.attention(qkv, nseq, L, H, dh, scale=scale)
        b.record()
        torch.cuda.synchronize()
        if base is None:
            base = out.clone()
        same = torch.equal(out, base)
        err = (out.float() - base.float()).abs().max().item()
        if reps > 1:
            ms = a.elapsed_time(b) / (reps - 1)
            res[v].append(ms)
            print(f"attention variant {v}: {ms:.4f} ms  {4.0 * L * L * dh * H * nseq / ms / 1e9:.1f} TFLOP/s  "
                  f"bit-identical to variant {variants[0]}: {same} (max |diff| {err:.2e})", flush=True)
K.set_option("attn_variant", 0)
for v, t in res.items():
    if t:
        print(f"variant {v}: best {min(t):.4f} ms  median {sorted(t)[len(t) // 2]:.4f} ms", flush=True)
