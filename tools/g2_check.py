"""Wide-row GEMM: elements off the fp32 reference by more than one bf16 step, per token-group
count and kernel version, at a bench-size M (debug aid)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

dev = "cuda"
M, Kd = int(sys.argv[1]) if len(sys.argv) > 1 else 49440, int(sys.argv[2]) if len(sys.argv) > 2 else 1536
g = torch.Generator(device="cpu").manual_seed(M + Kd)
a = torch.randn(M, Kd, generator=g).to(dev, torch.bfloat16)
w = (torch.randn(384, Kd, generator=g) / Kd ** 0.5).to(dev, torch.bfloat16)
b = torch.randn(384, generator=g).to(dev)
ref = a.float() @ w.float().t() + b
step = torch.exp2(torch.floor(torch.log2(ref.abs().clamp_min(1e-30))) - 7)
wp = K.gemm256_pack(w)
for var in (0, 4):
    for G in (8, 7, 6, 5, 4):
        K.set_option("g2_variant", var)
        K.set_option("g2_groups", G)
        outs = [K.gemm256(a, wp, 384, bias=b) for _ in range(3)]
        bad = [(o.float() - ref).abs() > step + 1e-4 * (1 + ref.abs()) for o in outs]
        nb = [int(x.sum()) for x in bad]
        rows = bad[0].any(1).nonzero().flatten()
        print(f"variant {var} groups {G}: bad {nb}, runs equal {[torch.equal(outs[0], o) for o in outs[1:]]}, "
              f"bad rows {rows.numel()} first {rows[:8].tolist()} rows mod 32G {sorted(set((rows % (32 * G)).tolist()))[:12]}",
              flush=True)
K.set_option("g2_variant", 0)
K.set_option("g2_groups", 0)

# which K-step's contribution is wrong on the bad rows (G = 7)?
K.set_option("g2_groups", int(os.environ.get("G2C_G", 7)))
o = K.gemm256(a, wp, 384, bias=b)
K.set_option("g2_groups", 0)
e = o.float() - ref
bad = ((e.abs() > step + 1e-4 * (1 + ref.abs())).any(1)).nonzero().flatten()
nk = Kd // 64
af, wf = a.float(), w.float()
for r in bad[:10].tolist():
    c = torch.stack([af[r, 64 * k:64 * k + 64] @ wf[:, 64 * k:64 * k + 64].t() for k in range(nk)])   # [nk, 384]
    res = [((e[r] + c[k]).norm().item(), k, "missing") for k in range(nk)] + \
          [((e[r] - c[k]).norm().item(), k, "twice") for k in range(nk)]
    # stale: step k's contribution computed with row r's data from step j
    best = min(res)
    cols = (e[r].abs() > 0.05).nonzero().flatten()
    print(f"row {r} (tile row {r % 224}, wg {r // 224}): |e| {e[r].norm().item():.3f}, bad features {cols.numel()} "
          f"first {cols[:8].tolist()}, best single-step explanation {best}", flush=True)
