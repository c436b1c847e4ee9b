"""Micro-benchmark of the fused block tail (csrc/ffn.hip, snvrag_block_tail_forward) variants
at the bench shape (M = 512 haplotypes x 1030 tokens, d384).  One line per variant: average
launch time (HIP events on the launch stream), TFLOP/s of the algorithmic 18*M*D^2, and the
max |difference| from the default variant's output (same inputs)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

M, D = int(os.environ.get("GM_M", 512 * 1030)), 384
REPS = int(os.environ.get("REPS", 10))
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "1,0,4,5,6,7,8,9").split(",")]
dev, bf = "cuda", torch.bfloat16
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(M, D, device=dev, generator=g).to(bf)
att = (0.5 * torch.randn(M, D, device=dev, generator=g)).to(bf)
w_o = (torch.randn(D, D, device=dev, generator=g) / D ** 0.5).to(bf)
w1 = (torch.randn(4 * D, D, device=dev, generator=g) / D ** 0.5).to(bf)
w2 = (torch.randn(D, 4 * D, device=dev, generator=g) / (4 * D) ** 0.5)
b_o, b1, b2 = (0.1 * torch.randn(n, device=dev, generator=g) for n in (D, 4 * D, D))
one, zero = torch.ones(D, device=dev), torch.zeros(D, device=dev)
w2g, b2g, _ = K.fold_layernorm(w2, b2, torch.ones(4 * D, device=dev), torch.zeros(4 * D, device=dev), bf)
ws = K.ffn_pack(w1, w2g)
vec = K.ffn_vec(b1, b2g, w2g, one, zero)
wo_s = K.ffn_pre_pack(w_o)
flop = 18.0 * M * D * D
ref = None
for v in VARIANTS:
    os.environ["SNVRAG_FFN_VARIANT"] = str(v)
    xx = x.clone()
    K.block_tail_forward(att, xx, wo_s, b_o, one, zero, ws, vec)
    out = xx.float()
    if ref is None:
        ref = out
    xs = [x.clone() for _ in range(REPS)]
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(REPS):
        K.block_tail_forward(att, xs[i], wo_s, b_o, one, zero, ws, vec)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / REPS
    err = (out - ref).abs().max().item()
    print(f"variant {v}: {ms:.4f} ms  {flop / ms / 1e9:.1f} TFLOP/s  max|d| vs first {err:.3e}", flush=True)
    del xs
