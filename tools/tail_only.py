"""Run only the 32x32-MFMA block tail kernel (rocprofv3 PMC passes); TAIL_FFN=1: the FFN-only entry."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

M, D = int(os.environ.get("GM_M", 512 * 1030)), 384
dev, bf = "cuda", torch.bfloat16
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(M, D, device=dev, generator=g).to(bf)
att = (0.5 * torch.randn(M, D, device=dev, generator=g)).to(bf)
w_o = (torch.randn(D, D, device=dev, generator=g) / D ** 0.5).to(bf)
w1 = (torch.randn(4 * D, D, device=dev, generator=g) / D ** 0.5).to(bf)
w2 = (torch.randn(D, 4 * D, device=dev, generator=g) / (4 * D) ** 0.5)
one, zero = torch.ones(D, device=dev), torch.zeros(D, device=dev)
w2g, b2g, _ = K.fold_layernorm(w2, zero, torch.ones(4 * D, device=dev), torch.zeros(4 * D, device=dev), bf)
ts = K.tail_pack(w_o, w1, w2g)
vec = K.ffn_vec(torch.zeros(4 * D, device=dev), b2g, w2g, one, zero)
out = torch.empty_like(x)
for _ in range(int(os.environ.get("REPS", 3))):
    if os.environ.get("TAIL_FFN"):
        K.tail_ffn_forward(x, ts, vec, out=out)
    else:
        K.tail_forward(att, x, ts, zero, one, zero, vec)
torch.cuda.synchronize()
print("ok")
