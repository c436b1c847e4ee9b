"""CPU replay of the r4 two-rank test's retrieval (tests/test_gpu_ddp.py
test_train_main_two_ranks_global_metrics_and_early_stop: --synthetic 8, 300 sites, 1 window, 40 panel
samples = 80 haplotypes, d128/L2, k = 4, lr 0, dropout 0) through the ORACLE, to find what can move
a sample's neighbours between runs.

For the train datasets of epochs 0 and 1 (the CSV's epochs 1 and 2) it reports per query:
  * the tie structure at the k-th neighbour of the canonical (distance, index) order — exact ties
    that straddle k are where any perturbation of the distances picks a different neighbour;
  * the kNN under the r4 range partitions of knn_scan (one process: 80 refs; two ranks: 40 per
    shard; scan_parts of r4 and r5) — exact per-range top-k + merge, which must equal the global
    top-k (partition invariance);
  * the plain LUT (binary Delta, the fast table path) against the exact-offset LUT
    (u = (W + A_q) - A_r with A_q = A_r = the window's AF embedding: the path a stale panel
    snapshot takes) — both in the device's f32 arithmetic (oracle/lut_f32.c).
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "rag-snvbert_amd")]
from oracle import knn_np, model_np  # noqa: E402
from src.dataset.synthetic import make_rag_dataset  # noqa: E402
from src.model import build_model  # noqa: E402

K = 4


def r4_parts(n_ref):
    p = (n_ref + 2047) // 2048
    return min(256, max(p, (n_ref + 63) // 64))


def partitioned_knn(codes, dq, k, n_parts, r0=0):
    n = codes.shape[0]
    rng = ((n + n_parts - 1) // n_parts + 15) // 16 * 16
    keys = []
    for a in range(0, n, rng):
        i, d = knn_np.knn(codes[a:a + rng], dq, k)
        keys.append(np.where(i >= 0, knn_np.pack_key(d, i + a + r0), np.uint64(~np.uint64(0))))
    return np.stack(keys)


def main():
    np.random.seed(0)                                  # train_embedding_rag.main seeds before build_data
    ds, vocab = make_rag_dataset(8, 300, 1, 40, seed=0, name="train")
    torch.manual_seed(0)
    m = build_model(len(vocab), 128, 2, 4, dropout=0.0)
    sd = {k: v.detach().float().numpy() for k, v in m.state_dict().items()}
    W = sd["bert.embedding.tokenizer.weight"]
    codes = ds.ref_alleles[0].astype(np.uint8)         # [80, 300]
    n = codes.shape[1]
    A = model_np.af_embedding(ds.ref_af_windows[0][None].astype(np.float32), sd)[0].astype(np.float32)
    for epoch in (0, 1):
        if epoch > 0:
            ds.regenerate_masks(epoch)
        ds.current_epoch = epoch
        items = [ds[i] for i in range(8)]
        tok = np.concatenate([np.stack([np.asarray(it["hap_1"]) for it in items]),
                              np.stack([np.asarray(it["hap_2"]) for it in items])]).astype(np.int64)
        sm = np.asarray(ds.window_masks[0][1:1 + n], np.uint8)
        dq_p, _ = knn_np.quantize_lut(knn_np.lut_delta_f32(W, tok, sm), 2)
        dq_x, _ = knn_np.quantize_lut(knn_np.lut_delta_f32(W, tok, sm, Aq=A[None], aq_period=1, Ar=A), 2)
        Dp = knn_np.distances(codes, dq_p)
        ip, vp = knn_np.topk_exact(Dp, K)
        ix, _ = knn_np.knn(codes, dq_x, K)
        straddle = sum(int((Dp[q] == vp[q, K - 1]).sum() > (vp[q] == vp[q, K - 1]).sum()) for q in range(len(tok)))
        # partition invariance: one process (80 refs) and two shards (40 each), r4 and r5 part counts
        want = knn_np.pack_key(vp, ip)
        inv = []
        for parts in (r4_parts(80), 2, 5):
            inv.append(np.array_equal(knn_np.merge_partials(partitioned_knn(codes, dq_p, K, parts), K), want))
        shard = [partitioned_knn(codes[40 * r:40 * (r + 1)], dq_p, K, r4_parts(40), 40 * r) for r in range(2)]
        inv.append(np.array_equal(knn_np.merge_partials(np.concatenate(shard), K), want))
        diff = [q for q in range(len(tok)) if set(ip[q]) != set(ix[q])]
        print(f"epoch {epoch}: {len(tok)} queries, k = {K}: ties straddling the k-th neighbour in {straddle}; "
              f"partitions (r4 1-process, 2, 5 ranges, 2 shards) == global top-k: {inv}; plain vs exact-offset "
              f"LUT neighbour sets differ for {len(diff)} queries {diff}; mask sites {int(sm.sum())}/{n}", flush=True)


if __name__ == "__main__":
    main()
