"""Imputation data path on the host, against outputs of the REFERENCE (tests/golden/infer_c5*.npz,
made by tests/golden/make_golden.py `infer` / `infer256`: the reference InferDataset,
EmbeddingRAGInferDataset and the statements of infer_embedding_rag.py:129-203 run on the
same synthetic arrays).

  * items: hap tokens, the target-missing-site masks, AF/pos features, window/sample ids —
    bit-exact (dataset.py:780-900, embedding_rag_infer_dataset.py:226-248);
  * index windows: 510-site infer masks, complete panel tokens, panel AF (:100-159);
  * A14: the oracle's post-processing + geometry (oracle/data_np.py) applied to the
    reference model's batch outputs reproduces the reference's imputed arrays (1e-6) — the
    oracle the GPU kernel is tested against is pinned here.
"""

import numpy as np
import pytest

from conftest import load_golden


def _dataset(g, index_window_len=510):
    from src.dataset.synthetic import make_infer_dataset, POPS
    a = dict(ori_pos=g["ori_pos"], pos=g["pos"], vcf=g["vcf"], freq=g["freq"], pops=g["cfg"]["pops"],
             pop_to_idx={p: i for i, p in enumerate(POPS)},
             pos_to_idx={int(p): i for i, p in enumerate(g["ori_pos"])}, ref_gt=g["ref_gt"], ref_pos=g["ref_pos"])
    return make_infer_dataset(a, index_window_len=index_window_len)[0]


@pytest.mark.parametrize("case", ["infer_c5", "infer_c5_b256", "infer_c5_d384", "infer_c5_m10", "infer_c5_m90"])
def test_infer_index_windows_match_reference(case):
    g = load_golden(case)
    ds = _dataset(g)
    assert ds.window_count == 2 and len(ds) == 2 * g["cfg"]["n_samples"]
    np.testing.assert_array_equal(np.stack(ds.infer_masks), g["infer_masks"])
    np.testing.assert_array_equal(np.stack(ds.ref_af_windows), g["ref_af_windows"])
    if "ref_tokens_complete" in g:
        np.testing.assert_array_equal(np.stack(ds.ref_tokens_complete), g["ref_tokens_complete"])
    # the panel lacks some sites: the index windows hold fewer sites than 510
    assert min(len(s) for s in ds.index_sites) < 510
    from src.dataset.sampler import WindowMajorSampler
    np.testing.assert_array_equal(np.array(list(iter(WindowMajorSampler(ds)))), g["order"])


def test_infer_items_match_reference():
    g = load_golden("infer_c5")
    ds = _dataset(g)
    for i in range(len(ds)):
        it = ds[i]
        for key in ("hap_1", "hap_2", "mask", "window_idx", "sample_idx", "start_idx", "end_idx"):
            np.testing.assert_array_equal(it[key].numpy(), g[f"item_{key}"][i], err_msg=f"{key} item {i}")
        for key in ("af", "af_p", "pos", "ref", "het", "hom"):
            np.testing.assert_array_equal(it[key].numpy(), g[f"item_{key}"][i].astype(np.float32), err_msg=key)
        assert it["window_idx"].dim() == 0


def test_infer_aligned_windows_mask_missing_sites():
    """index_window_len = window_len: every item's mask is exactly its own missing sites."""
    g = load_golden("infer_c5")
    ds = _dataset(g, index_window_len=1020)
    from src.dataset.dataset import InferDataset
    base = InferDataset(ds.vocab, ds.vcf, ds.pos, ds.panel, ds.freq, {}, ds.pop_to_idx, ds.pos_to_idx)
    for i in range(len(ds)):
        np.testing.assert_array_equal(ds[i]["mask"].numpy(), base[i]["mask"].numpy())
        np.testing.assert_array_equal(ds[i]["hap_1"].numpy(), base[i]["hap_1"].numpy())
    w = 1
    n = ds.window_bounds(w)[1] - ds.window_bounds(w)[0]
    np.testing.assert_array_equal(ds.infer_masks[w][1:1 + n], ds.position_needed[1020:1020 + n])


def test_a14_oracle_pinned_to_reference_outputs():
    """softmax-again + genotype products (infer_embedding_rag.py:145-152) and the [W,S,L] ->
    [W*L,S] geometry (:165-203) of the oracle, on the reference model's own batch outputs."""
    from oracle import data_np
    g = load_golden("infer_c5")
    p1, p2, gt = data_np.infer_probs(g["batch_probs_h1"], g["batch_probs_h2"])
    n_var = len(g["ori_pos"])
    h1, h2, gtg, mask = data_np.infer_geometry(p1, p2, gt, g["item_mask"][g["order"]], 2, n_var, 1020)
    np.testing.assert_allclose(h1, g["hap1"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(h2, g["hap2"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(gtg, g["gt"], rtol=1e-6, atol=1e-6)
    np.testing.assert_array_equal(mask, g["mask"])
    from src.infer_embedding_rag import geometry
    for a, b in zip(geometry(p1, p2, gt, g["item_mask"][g["order"]], 2, n_var, 1020), (h1, h2, gtg, mask)):
        np.testing.assert_array_equal(a, b)


def _split_worker(rank, world, port, n_rows, q):
    import os
    import traceback
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from src.infer_embedding_rag import _gather_rows, rank_rows
        lo, hi = rank_rows(n_rows, rank, world)
        rows = torch.arange(lo, hi, dtype=torch.long)
        sizes = [rank_rows(n_rows, r, world)[1] - rank_rows(n_rows, r, world)[0] for r in range(world)]
        full = _gather_rows(torch.stack([rows, -rows], 1), sizes)
        q.put((rank, full.numpy()))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_rows,world", [(256, 3), (2, 3), (7, 2)])
def test_infer_rank_split_and_ordered_gather_gloo(n_rows, world):
    """The multi-rank inference plumbing (src/infer_embedding_rag.py run): contiguous slices of the
    window-major stream cover every row once in order (a rank may get none), and the ragged
    gather returns the rows in stream order on every rank."""
    import socket
    import torch.multiprocessing as mp
    from src.infer_embedding_rag import rank_rows
    cover = [i for r in range(world) for i in range(*rank_rows(n_rows, r, world))]
    assert cover == list(range(n_rows))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_split_worker, args=(r, world, port, n_rows, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(30)
    want = np.stack([np.arange(n_rows), -np.arange(n_rows)], 1)
    for r in range(world):
        assert not isinstance(got[r], str), got[r]
        np.testing.assert_array_equal(got[r], want)
