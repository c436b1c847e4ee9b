"""Where the persistent block tail (tailp_kernel) and tail_kernel differ: rows / tiles / features."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

D, dev, bf = 384, "cuda", torch.bfloat16
for M in (777, 128 * 300):
    g = torch.Generator(device="cpu").manual_seed(M)
    x = torch.randn(M, D, generator=g).to(dev, bf)
    att = (0.5 * torch.randn(M, D, generator=g)).to(dev, bf)
    w_o = (torch.randn(D, D, generator=g) / math.sqrt(D)).to(dev, bf)
    b_o = (0.1 * torch.randn(D, generator=g)).to(dev)
    g1, be1 = (1 + 0.2 * torch.randn(D, generator=g)).to(dev), (0.1 * torch.randn(D, generator=g)).to(dev)
    w1 = (torch.randn(4 * D, D, generator=g) / math.sqrt(D)).to(dev, bf)
    w2 = (torch.randn(D, 4 * D, generator=g) / math.sqrt(4 * D)).to(dev)
    b1, b2 = torch.randn(4 * D, generator=g).to(dev), torch.randn(D, generator=g).to(dev)
    gf, bff = (1 + 0.2 * torch.randn(4 * D, generator=g)).to(dev), (0.1 * torch.randn(4 * D, generator=g)).to(dev)
    g2, be2 = (1 + 0.2 * torch.randn(D, generator=g)).to(dev), (0.1 * torch.randn(D, generator=g)).to(dev)
    w2g, b2g, _ = K.fold_layernorm(w2, b2, gf, bff, bf)
    vec = K.ffn_vec(b1, b2g, w2g, g2, be2)
    ts = K.tail_pack(w_o, w1, w2g)
    outs = []
    for persist in (1, 0, 1, 0):
        y = x.clone()
        with K.option("tail_persist", persist):
            K.tail_forward(att, y, ts, b_o, g1, be1, vec)
        outs.append(y)
    torch.cuda.synchronize()
    print(f"M={M}: p==p {torch.equal(outs[0], outs[2])} old==old {torch.equal(outs[1], outs[3])}")
    d = (outs[0].float() - outs[1].float()) != 0
    rows = d.any(1).nonzero().view(-1)
    print(f"  differing rows {rows.numel()} of {M}; per tile: {torch.bincount(rows // 128).tolist()[:40]}")
    print(f"  row-in-tile histogram: {torch.bincount(rows % 128, minlength=128).view(4, 32).sum(1).tolist()} (per wave)")
    print(f"  differing features per differing row: {d[rows].sum(1).float().mean().item() if rows.numel() else 0:.1f}")
    if rows.numel():
        r = rows[0].item()
        f = d[r].nonzero().view(-1)[:10].tolist()
        print(f"  row {r} features {f}: persist {outs[0][r, f].float().tolist()} old {outs[1][r, f].float().tolist()}")
