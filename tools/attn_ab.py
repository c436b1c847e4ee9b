"""A/B of the bf16 dh=32 attention kernels at the bench shape (512 sequences x 1030 tokens,
12 heads, prescaled Q): each variant selected by environment (read by the library per launch),
outputs compared bit for bit with the default kernel, times from CUDA events over REPS launches.
usage: VARIANTS="SNVRAG_ATTN_REGSTAGE=1" python tools/attn_ab.py"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

nseq, L, H, dh = int(os.environ.get("NSEQ", 512)), int(os.environ.get("L", 1030)), 12, 32
reps = int(os.environ.get("REPS", 10))
torch.manual_seed(0)
qkv = (torch.randn(nseq * L, 3 * H * dh, device="cuda") * float(os.environ.get("QKV_STD", 0.4))).to(torch.bfloat16)
qkv[:, :H * dh] = (qkv[:, :H * dh].float() * (math.log2(math.e) / math.sqrt(dh))).to(torch.bfloat16)
scale = 1.0 / math.log2(math.e)
flop = 4.0 * L * L * dh * H * nseq


def run(env):
    for kv in env:
        k, v = kv.split("=")
        os.environ[k] = v
    out = K.attention(qkv, nseq, L, H, dh, scale=scale)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        K.attention(qkv, nseq, L, H, dh, scale=scale)
    b.record()
    torch.cuda.synchronize()
    for kv in env:
        del os.environ[kv.split("=")[0]]
    return out, a.elapsed_time(b) / reps


base, ms0 = run([])
print(f"default: {ms0:.4f} ms  {flop / ms0 / 1e9:.1f} TFLOP/s", flush=True)
for var in os.environ.get("VARIANTS", "SNVRAG_ATTN_REGSTAGE=1").split(";"):
    env = var.split()
    out, ms = run(env)
    same = torch.equal(out, base)
    print(f"{var}: {ms:.4f} ms  {flop / ms / 1e9:.1f} TFLOP/s  bit-identical={same}  "
          f"max|d|={(out.float() - base.float()).abs().max().item():.3g}", flush=True)
_, ms1 = run([])
print(f"default again: {ms1:.4f} ms", flush=True)
