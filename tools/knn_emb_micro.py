"""Micro-benchmark of the embedding-space distance GEMM (csrc/knn_emb.hip) at the C2 shape:
N = 10,000 panel haplotypes x 1030 tokens x D = 384 (bf16, 7.9 GB, packed tiles), Bq in {48, 96, 128};
split-K sweep.  HBM bytes per launch = N * K * 2 (+ the queries)."""
import sys
import time
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402
from src import native as N  # noqa: E402

n, L, D = 10_000, 1030, 384
Kd = L * D
E = torch.empty(n, Kd, device="cuda", dtype=torch.bfloat16)
for i in range(0, n, 1000):
    E[i:i + 1000].normal_()
rn = K.knn_emb_norms(E)
Et = K.knn_emb_pack(E)
for bq in (48, 96, 128):
    Q = torch.randn(bq, Kd, device="cuda").bfloat16()
    qn = K.knn_emb_norms(Q)
    auto = int(N.lib().snvrag_knn_emb_splits(n, Kd, bq))
    for sp in sorted({auto, 16, 24, 48, 64}):
        K.knn_emb_dist(Et, Q, rn, qn, splits=sp)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            K.knn_emb_dist(Et, Q, rn, qn, splits=sp)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        gbs = (n + bq) * Kd * 2 / (ms * 1e-3) / 1e9
        print(f"Bq {bq:4d} splits {sp:3d}{' (auto)' if sp == auto else '       '}: {ms:7.3f} ms  "
              f"{gbs:7.1f} GB/s  frac {gbs / 8000:.3f}  (scan + finish)", flush=True)
# scan alone vs reference
Q = torch.randn(48, Kd, device="cuda").bfloat16()
d = K.knn_emb_dist(K.knn_emb_pack(E[:2000]), Q, rn[:2000])
ref = (Q.float().pow(2).sum(1)[:, None] + rn[None, :2000] - 2 * (Q.float() @ E[:2000].float().T))
print("max |d - torch f32|", (d - ref).abs().max().item(), flush=True)
