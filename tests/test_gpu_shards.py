"""Sharded panel on the GPU (src/retrieval/shards.py, csrc/knn.hip).

  * the shard kernels in one process: ``panel_synth`` rows of a shard equal the full
    panel's rows; two shards' local top-k keys (global indices) merged by ``topk_merge``
    equal the whole-panel search bit for bit; the shards' ``neighbor_counts`` add up to
    the full counts (== numpy); ``rag_mean`` from counts == ``rag_mean`` from the panel rows;
  * the product path across processes: two ranks (gloo, tensors staged through the host,
    both ranks on the one GPU) run ``EmbeddingRAGDataset.process_batch_retrieval`` with the
    panel sharded 2-way and ragged per-rank batches, and the bench's sharded search — each
    rank's neighbours and neighbour means equal a single-process run on the whole panel.
"""

import os
import socket
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_shard_kernels_merge_counts_and_means():
    from src import kernels as K
    from src.retrieval import PanelIndex
    from src.retrieval.shards import kernel_ops
    rng = np.random.default_rng(2)
    N, S, k, L, D = 5000, 500, 16, 1030, 64
    af = torch.from_numpy(rng.beta(0.3, 3.0, S).astype(np.float32)).to(DEV)
    ref_af = torch.zeros(L, device=DEV)
    full = K.panel_synth(N, S, af, 9)
    cut = 1733                                               # not a multiple of any tile
    a = K.panel_synth(cut, S, af, 9, row0=0)
    b = K.panel_synth(N - cut, S, af, 9, row0=cut)
    torch.testing.assert_close(torch.cat([a, b]), full, rtol=0, atol=0)
    W = torch.from_numpy(rng.standard_normal((12, D)).astype(np.float32)).to(DEV)
    site_mask = torch.from_numpy((rng.random(S) < 0.4).astype(np.uint8)).to(DEV)
    codes_h = full.cpu().numpy()[:, :S]
    nq = 70
    tok = np.zeros((nq, L), np.int64)
    tok[:, 0], tok[:, S + 1] = 2, 3
    q = codes_h[rng.integers(0, N, nq)] ^ (rng.random((nq, S)) < 0.03)
    tok[:, 1:S + 1] = np.where(site_mask.cpu().numpy()[None] == 1, 4, 5 + q)
    tok = torch.from_numpy(tok).to(DEV)
    whole = PanelIndex(full, S, ref_af)
    idx_w, _, keys_w, _, _ = whole.search(tok, W, site_mask, k, return_keys=True)
    parts = []
    for codes, r0 in ((a, 0), (b, cut)):
        ops = kernel_ops(PanelIndex(codes, S, ref_af, ref_offset=r0, n_total=N), W, site_mask, k)
        parts.append(ops.keys(tok, None)[0])
    merged = K.topk_merge(torch.stack(parts), k)
    torch.testing.assert_close(merged, keys_w, rtol=0, atol=0)
    idx, _ = K.knn_decode(merged)
    torch.testing.assert_close(idx, idx_w, rtol=0, atol=0)
    ca = K.neighbor_counts(idx, a, 0)
    cb = K.neighbor_counts(idx, b, cut)
    cnt = ca + cb
    want = codes_h[idx.cpu().numpy()].sum(1)
    np.testing.assert_array_equal(cnt.cpu().numpy()[:, :S], want)
    assert int(cnt[:, S:].max()) == 0
    torch.testing.assert_close(cnt, K.neighbor_counts(idx, full, 0), rtol=0, atol=0)
    pe = torch.from_numpy(rng.standard_normal((L, D)).astype(np.float32)).to(DEV)
    Ar = torch.from_numpy(rng.standard_normal((L, D)).astype(np.float32)).to(DEV)
    for dt in (torch.float32, torch.bfloat16):
        m_idx = K.rag_mean(idx, full, S, W, pe, Ar, L, dt)
        m_cnt = K.rag_mean(idx, full[:1], S, W, pe, Ar, L, dt, counts=cnt)
        torch.testing.assert_close(m_cnt, m_idx, rtol=0, atol=0)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _reference_run():
    """Single process, whole panel: per-rank batches' neighbours and means."""
    from src.dataset.synthetic import make_rag_dataset
    from src.engine import engine_for
    from src.model import build_model
    torch.manual_seed(0)
    np.random.seed(0)      # the construction-time window masks draw from the global RNG
    ds, vocab = make_rag_dataset(n_samples=7, n_sites=300, n_windows=2, n_ref_samples=40, seed=3)
    m = build_model(len(vocab), 64, 1, 4).to(DEV).eval()
    engine_for(m).set_dtype(torch.float32)
    return ds, m


def _batches(ds, rank):
    from src.dataset.embedding_rag_dataset import embedding_rag_collate_fn
    # ragged: rank 0 gets 5 items spanning both windows, rank 1 gets 2 items of window 1
    items = [0, 1, 2, 3, 5] if rank == 0 else [7, 9]
    return embedding_rag_collate_fn([ds[i] for i in items])


def _rank_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        root = os.path.join(os.path.dirname(__file__), "..")
        sys.path[:0] = [root, os.path.join(root, "rag-snvbert_amd")]
        from src.retrieval.shards import PanelShard
        ds, m = _reference_run()
        ds.set_panel_shard(PanelShard.current())
        b = ds.process_batch_retrieval(_batches(ds, rank), m.bert.embedding, DEV, k_retrieve=6)
        res = dict(idx1=b["rag_idx_h1"].cpu().numpy(), idx2=b["rag_idx_h2"].cpu().numpy(),
                   mean=b["rag_mean"].float().cpu().numpy())
        # the bench's sharded search over a hash-generated panel
        import bench
        from src.dataset.vocab import WordVocab
        from src.dataset import synthetic
        args = SimpleNamespace(batch=3 + rank, n_ref=3000, window=256, level=4)
        from src.engine import engine_for
        wl = bench.build_workload(args, torch.device(DEV), WordVocab(synthetic.POPS), rank,
                                  shard=PanelShard.current())
        idx, counts = bench.make_search(wl, engine_for(m), 8)()
        res.update(bench_idx=idx.cpu().numpy(), bench_counts=counts.cpu().numpy())
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_retrieval_two_ranks_matches_single_process():
    import bench
    from src.dataset.vocab import WordVocab
    from src.dataset import synthetic
    from src.engine import engine_for
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=280) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    ds, m = _reference_run()
    for r in range(2):
        b = ds.process_batch_retrieval(_batches(ds, r), m.bert.embedding, DEV, k_retrieve=6)
        np.testing.assert_array_equal(got[r]["idx1"], b["rag_idx_h1"].cpu().numpy())
        np.testing.assert_array_equal(got[r]["idx2"], b["rag_idx_h2"].cpu().numpy())
        np.testing.assert_array_equal(got[r]["mean"], b["rag_mean"].float().cpu().numpy())
        args = SimpleNamespace(batch=3 + r, n_ref=3000, window=256, level=4)
        wl = bench.build_workload(args, torch.device(DEV), WordVocab(synthetic.POPS), r)
        idx, _ = bench.make_search(wl, engine_for(m), 8)()
        np.testing.assert_array_equal(got[r]["bench_idx"], idx.cpu().numpy())
        codes = wl.index.codes.cpu().numpy()
        np.testing.assert_array_equal(got[r]["bench_counts"], codes[idx.cpu().numpy()].sum(1))


# ------------------------------------------------------------------ 8 ranks on the one GPU
W8_ITEMS = [[0, 1, 2], [5], [3, 9, 11, 4], [15], [7, 8], [10], [6, 12, 13], [14]]   # ragged, both windows


def _batches8(ds, rank):
    from src.dataset.embedding_rag_dataset import embedding_rag_collate_fn
    return embedding_rag_collate_fn([ds[i] for i in W8_ITEMS[rank]])


def _reference_run8():
    from src.dataset.synthetic import make_rag_dataset
    from src.engine import engine_for
    from src.model import build_model
    torch.manual_seed(0)
    np.random.seed(0)
    ds, vocab = make_rag_dataset(n_samples=16, n_sites=200, n_windows=2, n_ref_samples=45, seed=4)
    m = build_model(len(vocab), 64, 1, 4).to(DEV).eval()
    engine_for(m).set_dtype(torch.float32)
    return ds, m


def _rank_worker8(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        root = os.path.join(os.path.dirname(__file__), "..")
        sys.path[:0] = [root, os.path.join(root, "rag-snvbert_amd")]
        from src.retrieval.shards import PanelShard
        from src.engine import engine_for
        ds, m = _reference_run8()
        ds.set_panel_shard(PanelShard.current())
        b = ds.process_batch_retrieval(_batches8(ds, rank), m.bert.embedding, DEV, k_retrieve=5)
        res = dict(idx1=b["rag_idx_h1"].cpu().numpy(), idx2=b["rag_idx_h2"].cpu().numpy(),
                   mean=b["rag_mean"].float().cpu().numpy())
        import bench
        from src.dataset.vocab import WordVocab
        from src.dataset import synthetic
        args = SimpleNamespace(batch=1 + rank % 3, n_ref=2500, window=192, level=4)
        wl = bench.build_workload(args, torch.device(DEV), WordVocab(synthetic.POPS), rank,
                                  shard=PanelShard.current())
        idx, counts = bench.make_search(wl, engine_for(m), 8)()
        res.update(bench_idx=idx.cpu().numpy(), bench_counts=counts.cpu().numpy())
        q.put((rank, res))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(400)
def test_sharded_retrieval_eight_ranks_one_gpu_matches_single_process():
    """configs[3]'s 8-way panel shard at tiny size: 8 gloo ranks on the one GPU run the HIP
    shard kernels (local scan with global indices, 8-list topk_merge, neighbour counts
    all-reduce) under the product path — ragged batches over two windows — and every rank's
    neighbours and means equal one process on the whole panel."""
    import bench
    from src.dataset.vocab import WordVocab
    from src.dataset import synthetic
    from src.engine import engine_for
    world = 8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_worker8, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=380) for _ in ps)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for r in range(world):
        assert isinstance(got[r], dict), got[r]
    ds, m = _reference_run8()
    for r in range(world):
        b = ds.process_batch_retrieval(_batches8(ds, r), m.bert.embedding, DEV, k_retrieve=5)
        np.testing.assert_array_equal(got[r]["idx1"], b["rag_idx_h1"].cpu().numpy())
        np.testing.assert_array_equal(got[r]["idx2"], b["rag_idx_h2"].cpu().numpy())
        np.testing.assert_array_equal(got[r]["mean"], b["rag_mean"].float().cpu().numpy())
        args = SimpleNamespace(batch=1 + r % 3, n_ref=2500, window=192, level=4)
        wl = bench.build_workload(args, torch.device(DEV), WordVocab(synthetic.POPS), r)
        idx, _ = bench.make_search(wl, engine_for(m), 8)()
        np.testing.assert_array_equal(got[r]["bench_idx"], idx.cpu().numpy())
        codes = wl.index.codes.cpu().numpy()
        np.testing.assert_array_equal(got[r]["bench_counts"], codes[idx.cpu().numpy()].sum(1))
