"""World-size-2 and -8 gloo tests of the sharded retrieval (src/retrieval/shards.py):
each rank owns a contiguous range of the panel, computes its exact local top-k with GLOBAL
indices, the partial key lists are all-gathered and merged, and the neighbours' per-site
alt-allele counts are all-reduced — results must equal the single-shard canonical top-k
and the full-panel counts bit for bit.  The product plumbing (``sharded_neighbours``,
``all_gather_rows`` with ragged per-rank query counts, ``batch_windows``) runs as shipped;
only its compute steps (LUT + scan, merge, decode, counts) are the oracle's on the CPU —
on the GPU the same plumbing drives knn_scan / topk_merge / neighbor_counts over RCCL."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import knn_np


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _case(seed=3, n_ref=301, n_sites=96, nq=6, k=8):
    rng = np.random.default_rng(seed)
    codes = (rng.random((n_ref, n_sites)) < 0.2).astype(np.uint8)
    codes[:20] = codes[20:40]                          # exact duplicates -> distance ties
    dq = rng.integers(-300, 300, size=(nq, n_sites)).astype(np.int32)
    return codes, dq, k


def _local_keys(codes, dq, k, r0):
    D = knn_np.distances(codes, dq)
    I, V = knn_np.topk_exact(D, k)
    return np.where(I >= 0, knn_np.pack_key(V, I + r0), np.uint64(~np.uint64(0)))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
        from src.retrieval.shards import sharded_search
        codes, dq, k = _case()
        bounds = np.linspace(0, codes.shape[0], world + 1).astype(int)
        r0, r1 = bounds[rank], bounds[rank + 1]
        local = torch.from_numpy(_local_keys(codes[r0:r1], dq, k, r0).view(np.int64)).view(torch.uint64)

        def merge(g, kk):
            return torch.from_numpy(knn_np.merge_partials(g.view(torch.int64).numpy().view(np.uint64), kk)
                                    .view(np.int64)).view(torch.uint64)

        out = sharded_search(local, k, merge_fn=merge)
        q.put((rank, out.view(torch.int64).numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world", [2, 8])
def test_sharded_topk_equals_single_shard(world):
    codes, dq, k = _case()
    want = _local_keys(codes, dq, k, 0).view(np.int64)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=200) for _ in ps)
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    for r in range(world):
        np.testing.assert_array_equal(got[r], want)


# ---------------------------------------------------------------------------- product plumbing
# ragged per-rank query counts (world 8: one rank without queries)
QUERIES = {2: (5, 3), 8: (5, 3, 1, 4, 0, 2, 6, 3)}
WINDOWS = {2: ([3, 1], [1, 4]), 8: ([3, 1], [1, 4], [1], [], [7], [3], [1, 3], [0])}


def _plumbing_case(world=2, seed=5, n_ref=203, n_sites=80, k=6):
    rng = np.random.default_rng(seed)
    codes = (rng.random((n_ref, n_sites)) < 0.25).astype(np.uint8)
    codes[:10] = codes[50:60]                          # ties across the shard boundary
    codes[120:130] = codes[20:30]                      # (world 8: ties across several shards)
    W = rng.standard_normal((11, 16)).astype(np.float32)
    site_mask = (rng.random(n_sites) < 0.3).astype(np.uint8)
    L = n_sites + 2
    toks = []
    for nq in QUERIES[world]:
        t = np.zeros((nq, L), np.int64)
        t[:, 0], t[:, -1] = 2, 3
        src = codes[rng.integers(0, n_ref, nq)] ^ (rng.random((nq, n_sites)) < 0.05)
        t[:, 1:-1] = np.where(site_mask[None] == 1, 4, 5 + src)
        toks.append(t)
    return codes, W, site_mask, toks, k


def _oracle_ops(codes_local, r0, W, site_mask, k):
    from src.retrieval.shards import ShardOps

    def keys(tok_all, af_all):
        assert af_all is None
        dq, e = knn_np.quantize_lut(knn_np.lut_delta(W, tok_all.numpy(), None, site_mask), 2)
        return torch.from_numpy(_local_keys(codes_local, dq, k, r0).view(np.int64)), torch.from_numpy(e), None

    def merge(g, kk):
        return torch.from_numpy(knn_np.merge_partials(g.numpy().view(np.uint64), kk).view(np.int64))

    def decode(keys, exps, consts):
        kk = keys.numpy().view(np.uint64)
        idx = (kk & np.uint64(0xFFFFFFFF)).astype(np.int64)
        d = (kk >> np.uint64(32)).astype(np.int64) - (1 << 30)
        return torch.from_numpy(idx), torch.from_numpy(d.astype(np.float32))

    def counts(idx):
        i = idx.numpy() - r0
        own = (i >= 0) & (i < codes_local.shape[0])
        c = np.zeros((i.shape[0], codes_local.shape[1]), np.uint8)
        for q in range(i.shape[0]):
            for j in range(i.shape[1]):
                if own[q, j]:
                    c[q] += codes_local[i[q, j]]
        return torch.from_numpy(c)

    return ShardOps(keys=keys, merge=merge, decode=decode, counts=counts)


def _plumbing_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
        from src.retrieval.shards import PanelShard, batch_windows, sharded_neighbours
        codes, W, site_mask, toks, k = _plumbing_case(world)
        shard = PanelShard.current()
        r0, r1 = shard.bounds(codes.shape[0])
        ops = _oracle_ops(codes[r0:r1], r0, W, site_mask, k)
        idx, d, cnt = sharded_neighbours(torch.from_numpy(toks[rank]), k, ops, None, shard.group)
        wins = batch_windows(WINDOWS[world][rank], shard.group)
        q.put((rank, idx.numpy().copy(), cnt.numpy().copy(), wins))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(240)
@pytest.mark.parametrize("world", [2, 8])
def test_sharded_neighbours_product_plumbing(world):
    codes, W, site_mask, toks, k = _plumbing_case(world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_plumbing_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = {}
    for _ in ps:
        r, idx, cnt, wins = q.get(timeout=200)
        got[r] = (idx, cnt, wins)
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    want_w = sorted({w for ws in WINDOWS[world] for w in ws})
    for r in range(world):
        idx, cnt, wins = got[r]
        assert wins == want_w
        assert idx.shape == (QUERIES[world][r], k)
        if QUERIES[world][r] == 0:
            continue
        dq, _ = knn_np.quantize_lut(knn_np.lut_delta(W, toks[r], None, site_mask), 2)
        want_i, _ = knn_np.knn(codes, dq, k)
        np.testing.assert_array_equal(idx, want_i)
        np.testing.assert_array_equal(cnt, codes[want_i].sum(1).astype(np.uint8))
