"""GPU tests of the imputation entry point (src/infer_embedding_rag.py): the device
post-processing kernel vs the oracle restatement of infer_embedding_rag.py:145-152
(1e-6), and an end-to-end synthetic run (retrieval + forward + post-processing +
geometry + writers) at the C5 mask sweep end points."""

import numpy as np
import pytest
import torch

from oracle import data_np

pytestmark = pytest.mark.gpu


def test_infer_post_kernel_vs_oracle():
    from src import kernels as K
    rng = np.random.default_rng(0)
    a = rng.random((3, 1030, 2)).astype(np.float32)
    b = rng.random((3, 1030, 2)).astype(np.float32)
    a /= a.sum(-1, keepdims=True)
    b /= b.sum(-1, keepdims=True)
    p1, p2, gt = K.infer_post(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda())
    o1, o2, og = data_np.infer_probs(a, b)
    np.testing.assert_allclose(p1.cpu().numpy(), o1, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(p2.cpu().numpy(), o2, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(gt.cpu().numpy(), og, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("rate", [0.1, 0.9])
def test_infer_entry_synthetic(tmp_path, rate):
    """C5 sweep end points through the CLI (aligned index windows: the mask is exactly the
    target-missing sites, so its mean is the sweep rate)."""
    from src.infer_embedding_rag import infer
    res = infer(["--synthetic", "6", "--synthetic_sites", "2040", "--synthetic_ref", "24", "-d", "64", "-l", "2",
                 "-a", "2", "-b", "4", "--k_retrieve", "3", "--mask_rate", str(rate), "--index_window_len", "1020",
                 "-o", str(tmp_path)])
    h1, gt, mask = res["h1"], res["gt"], res["mask"]
    assert h1.shape == (2040, 6) and gt.shape == (2040, 6, 4) and mask.shape == (2040, 6)
    assert np.isfinite(h1).all() and (h1 > 0).all() and (h1 < 1).all()
    np.testing.assert_allclose(gt.sum(-1), 1.0, rtol=1e-5)
    assert abs(mask.mean() - rate) < 0.05
    assert (mask == mask[:, :1]).all()                       # the missing sites are the same for every sample
    vcf = (tmp_path / "imputed.vcf").read_text().splitlines()
    body = [l for l in vcf if not l.startswith("#")]
    assert len(body) == int(mask[:, 0].sum()) and body[0].count("\t") == 9 + 6 - 1


def _fixture_run(case, dtype):
    from conftest import golden_state_dict, load_golden
    from src.engine import engine_for
    from src.infer_embedding_rag import run
    from src.model import build_model
    from test_infer_cpu import _dataset
    g = load_golden(case)
    cfg = g["cfg"]
    sd = golden_state_dict(cfg)
    m = build_model(cfg["vocab"], cfg["d"], cfg["layers"], cfg["heads"])
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    m = m.to("cuda").eval()
    engine_for(m).set_dtype(dtype)
    ds = _dataset(g)
    return g, cfg, ds, run(ds, m, torch.device("cuda"), cfg["batch_size"], cfg["k"])


@pytest.mark.parametrize("case,dtype", [("infer_c5", torch.float32), ("infer_c5", torch.bfloat16),
                                        ("infer_c5_b256", torch.float32), ("infer_c5_b256", torch.bfloat16),
                                        ("infer_c5_d384", torch.float32), ("infer_c5_d384", torch.bfloat16),
                                        ("infer_c5_m10", torch.float32), ("infer_c5_m90", torch.float32),
                                        ("infer_c5_m90", torch.bfloat16)])
def test_infer_matches_reference_fixture(case, dtype):
    """The whole imputation path (EmbeddingRAGInferDataset items, 510-site index windows,
    process_batch_retrieval on the HBM index, forward, device post-processing, geometry) vs
    the reference run on the same arrays (tests/golden/make_golden.py run_infer_case): the
    d64/L2 cases at batch 4 and 256, the v18 shape d384/L12/H12, and the C5 sweep end points
    (10 % / 90 % of the panel sites missing from the target), in f32 and bf16.
    Neighbours: equal top-k sets wherever the reference's k-th/(k+1)-th distance margin is
    not a tie (> 1e-3); imputed probabilities of the sample-windows whose neighbours are
    unambiguous: f32 1e-4 (1e-3 against the float16-stored fixtures), bf16 2e-2 (3e-2 at
    d384/L12); masks bit-exact.  The tied sample-windows are covered by
    test_infer_tied_rows_vs_oracle."""
    g, cfg, ds, res = _fixture_run(case, dtype)
    k, S = cfg["k"], cfg["n_samples"]
    clear = (g["kth_margin_h1"] > 1e-3) & (g["kth_margin_h2"] > 1e-3)
    assert clear.mean() > 0.6                               # (128 samples copied from 48 panel haplotypes: ties)
    for h in ("1", "2"):
        got = np.sort(res[f"idx{h}"], 1)[clear]
        np.testing.assert_array_equal(got, np.sort(g[f"I_h{h}"], 1)[clear])
    np.testing.assert_array_equal(res["mask"], g["mask"])
    # sampler row r = window r // S, sample r % S -> geometry rows [1020 w, 1020 w + 1020), column s
    ok = np.zeros((len(g["ori_pos"]), S), bool)
    for r in np.nonzero(clear)[0]:
        w, s = divmod(int(r), S)
        ok[1020 * w:1020 * (w + 1), s] = True
    tol = 1e-4 if dtype == torch.float32 else (3e-2 if cfg["layers"] > 2 else 2e-2)
    if g["hap1"].dtype == np.float16:
        tol = max(tol, 1e-3)
    for h in ("1", "2"):
        np.testing.assert_allclose(res[f"h{h}"][ok], g[f"hap{h}"].astype(np.float32)[ok], atol=tol, rtol=0)
    if "gt" in g:
        np.testing.assert_allclose(res["gt"][ok], g["gt"][ok], atol=2 * tol, rtol=0)


@pytest.mark.parametrize("case", ["infer_c5_b256", "infer_c5_m90"])
def test_infer_tied_rows_vs_oracle(case):
    """The sample-windows the fixture test above leaves out (the reference's k-th neighbour
    distance ties the (k+1)-th: its FAISS order picks one of the tied haplotypes arbitrarily).
    For EVERY row: our neighbours are tie-equivalent to the reference's — the multisets of exact
    (float64) squared distances in the reference's own index embedding space are equal
    (embedding_rag_infer_dataset.py:164-181, :274-285) — and our imputed p(alt) equals the
    oracle (oracle/model_np.forward + data_np.infer_probs, infer_embedding_rag.py:141-152) run
    on OUR neighbours within 1e-4 (f32).  Together with the fixture test this covers 100 % of
    the sample-windows."""
    from conftest import golden_state_dict, load_golden
    from oracle import data_np, model_np
    from src.dataset.sampler import WindowMajorSampler
    g, cfg, ds, res = _fixture_run(case, torch.float32)
    k = cfg["k"]
    sd = golden_state_dict(cfg)
    sd = {kk: np.asarray(v, np.float32) for kk, v in sd.items()}
    order = list(iter(WindowMajorSampler(ds)))
    tied = np.nonzero(~((g["kth_margin_h1"] > 1e-3) & (g["kth_margin_h2"] > 1e-3)))[0]
    assert len(tied) > 0
    check_rows = sorted(set(tied.tolist()) | {0, len(order) - 1})
    for r in check_rows:
        it = ds[order[r]]
        w = int(it["window_idx"])
        ref_tok = np.asarray(ds.ref_tokens_complete[w]).astype(np.int64)
        ref_af = np.asarray(ds.ref_af_windows[w], np.float32)
        masked = ref_tok.copy()
        masked[:, np.asarray(ds.infer_masks[w]) == 1] = 4
        e_ref = model_np.embed(masked, np.broadcast_to(ref_af, masked.shape), sd).astype(np.float64)
        af = it["af"].numpy()[None]
        for h, ours, theirs in (("1", res["idx1"][r], g["I_h1"][r]), ("2", res["idx2"][r], g["I_h2"][r])):
            e_q = model_np.embed(it[f"hap_{h}"].numpy()[None], af, sd).astype(np.float64)[0]
            d = ((e_ref - e_q[None]) ** 2).sum((1, 2))
            np.testing.assert_allclose(np.sort(d[ours]), np.sort(d[theirs]), rtol=1e-6,
                                       err_msg=f"row {r} h{h}: not tie-equivalent")
        xo = {key: it[key].numpy()[None] for key in ("hap_1", "hap_2", "af", "af_p", "pos", "ref", "het", "hom")}
        xo["rag_mean_h1"] = model_np.rag_mean(ref_tok, res["idx1"][r][None], ref_af, sd)
        xo["rag_mean_h2"] = model_np.rag_mean(ref_tok, res["idx2"][r][None], ref_af, sd)
        o = model_np.forward(xo, sd, cfg["layers"], cfg["heads"])
        p1, p2, _ = data_np.infer_probs(o["probs_h1"], o["probs_h2"])
        np.testing.assert_allclose(res["batch_h1"][r], p1[0], atol=1e-4, rtol=0, err_msg=f"row {r}")
        np.testing.assert_allclose(res["batch_h2"][r], p2[0], atol=1e-4, rtol=0, err_msg=f"row {r}")


# ---------------------------------------------------------------- several ranks (configs[4]) --
def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _infer_rank_worker(rank, world, port, mode, arg, q):
    """One rank of a gloo group, every rank on cuda:0: ``mode`` "fixture" runs ``run`` on a golden
    case, "cli" runs the ``infer`` entry point (WORLD_SIZE / RANK from the environment)."""
    import os
    import sys
    import traceback
    import faulthandler
    faulthandler.dump_traceback_later(200, exit=True)
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.join(here, "..")
    sys.path[:0] = [root, os.path.join(root, "rag-snvbert_amd"), here]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK="0")
    import torch.distributed as dist
    try:
        torch.cuda.set_device(0)
        if mode == "fixture":
            dist.init_process_group("gloo", rank=rank, world_size=world)
            case, dt = arg
            _, _, _, res = _fixture_run(case, getattr(torch, dt))
        else:
            from src.infer_embedding_rag import infer
            res = infer(arg + ["--dist_backend", "gloo"])
        q.put((rank, {k: v for k, v in res.items() if isinstance(v, np.ndarray)} | {"seconds": res["seconds"]}))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run_ranks(world, mode, arg):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_infer_rank_worker, args=(r, world, port, mode, arg, q)) for r in range(world)]
    for p in ps:
        p.start()
    try:
        got = dict(q.get(timeout=250) for _ in ps)
    finally:
        for p in ps:
            p.join(30)
            if p.is_alive():
                p.kill()
                p.join(10)
    for r, v in got.items():
        assert not isinstance(v, str), f"rank {r}:\n{v}"
    assert all(p.exitcode == 0 for p in ps)
    return got


_KEYS = ("h1", "h2", "gt", "mask", "idx1", "idx2", "batch_h1", "batch_h2", "batch_mask")


@pytest.mark.timeout(400)
@pytest.mark.parametrize("case,dtype,world", [("infer_c5_b256", "bfloat16", 3), ("infer_c5_m90", "float32", 2)])
def test_infer_ranks_match_single_process(case, dtype, world):
    """configs[4] across ranks: the panel replicated, each rank imputing a contiguous slice of the
    window-major stream (3 ranks split the 256 sample-windows 85/85/86, across the window
    boundary), the outputs gathered in stream order — every rank's arrays equal the single-process
    run on the same fixture bit for bit (reference loop: infer_embedding_rag.py:129-203)."""
    got = _run_ranks(world, "fixture", (case, dtype))
    _, _, _, one = _fixture_run(case, getattr(torch, dtype))
    for r in range(world):
        for k in _KEYS:
            np.testing.assert_array_equal(got[r][k], one[k], err_msg=f"rank {r} {k}")


@pytest.mark.timeout(400)
def test_infer_cli_two_ranks_writes_single_process_output(tmp_path):
    """The entry point under WORLD_SIZE = 2: rank 0 writes imputed.npz / imputed.vcf identical to
    a single-process run's; rank 1 writes nothing."""
    args = ["--synthetic", "6", "--synthetic_sites", "2040", "--synthetic_ref", "24", "-d", "64", "-l", "2", "-a", "2",
            "-b", "4", "--k_retrieve", "3", "--mask_rate", "0.5", "--index_window_len", "1020"]
    _run_ranks(2, "cli", args + ["-o", str(tmp_path / "ddp")])
    from src.infer_embedding_rag import infer
    infer(args + ["-o", str(tmp_path / "one")])
    a, b = np.load(tmp_path / "ddp" / "imputed.npz"), np.load(tmp_path / "one" / "imputed.npz")
    for k in b.files:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert (tmp_path / "ddp" / "imputed.vcf").read_text() == (tmp_path / "one" / "imputed.vcf").read_text()


@pytest.mark.timeout(300)
def test_infer_cli_loads_reference_pickled_module(tmp_path):
    """``--check_point`` given the reference trainer's own checkpoint object (a pickled
    BERTFoundationModel, tests/golden/ref_module_tiny.pth, infer_embedding_rag.py:93-103) imputes
    exactly what the converted state_dict file does, and not what the random-init weights do."""
    import os
    from src.infer_embedding_rag import infer
    from src.model.checkpoint import load_state_dict_any
    pth = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_module_tiny.pth")
    torch.save(load_state_dict_any(pth), tmp_path / "sd.pt")
    args = ["--synthetic", "4", "--synthetic_sites", "1020", "--synthetic_ref", "24", "-d", "64", "-l", "2", "-a", "2",
            "-b", "4", "--k_retrieve", "3", "--mask_rate", "0.5", "--no_vcf"]
    infer(args + ["-o", str(tmp_path / "pickled"), "--check_point", pth])
    infer(args + ["-o", str(tmp_path / "sd"), "--check_point", str(tmp_path / "sd.pt")])
    infer(args + ["-o", str(tmp_path / "init")])
    a, b, c = (np.load(tmp_path / n / "imputed.npz") for n in ("pickled", "sd", "init"))
    for k in b.files:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    assert not np.array_equal(a["hap1"], c["hap1"])
