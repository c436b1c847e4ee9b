"""World-size-2 gloo test of the sharded kNN exchange: each rank owns a
contiguous range of the panel, computes its exact local top-k with GLOBAL indices, the
partial key lists are all-gathered and merged — the result must equal the single-shard
canonical top-k bit for bit.  The local top-k and the merge are the oracle's here (CPU);
on the GPU the same exchange runs with knn_scan/topk_merge over RCCL."""

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


@pytest.mark.timeout(120)
def test_sharded_topk_equals_single_shard_world2():
    codes, dq, k = _case()
    want = _local_keys(codes, dq, k, 0).view(np.int64)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=100) for _ in ps)
    for p in ps:
        p.join(30)
        assert p.exitcode == 0
    for r in range(2):
        np.testing.assert_array_equal(got[r], want)
