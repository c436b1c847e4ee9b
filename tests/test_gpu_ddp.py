"""Data-parallel training across ranks on the real training graph (SURVEY.md §8e, configs[3]),
two ranks on the one GPU of the test box over gloo (host-staged collectives; the same code
issues RCCL collectives with one GPU per rank).

  * ``BERTTrainerWithValidationOptimized.train_step`` on a d128/L2 model with train-mode
    retrieval (the AF MLP then runs for the queries AND once per neighbour window group, so its
    parameters are used several times per step) and ``direct_weight_grads`` (Linear / LayerNorm
    backward adding dW straight into the flat gradient buffer), for a sharded and a replicated
    panel, dropout 0.  Asserted per step: every bucket's all-reduce is issued only after each of
    its parameters became final (its AccumulateGrad ran) and in bucket order on both ranks, also
    when the ranks hold different numbers of window groups; after the steps both ranks' weights
    are bitwise equal; the reduced gradient equals the sum of single-process gradients of the two
    ranks' batches (1e-5) and, for a one-window step, the single-process gradient of the union
    batch.
  * ``train_embedding_rag.main`` on two ranks: the epoch CSV rows (summed counts and losses
    over ranks) equal a single-process run with the global batch on the same data, both ranks
    stop early at the same epoch, and nothing hangs.

Reference semantics: pretrain_with_val_optimized.py:59-65 (DataParallel: one gradient of the
summed loss over the global batch), :235-245 (clip + step), :362-422 / :490-522 (epoch metrics,
early stopping)."""

import csv
import os
import socket
import sys
import traceback

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
DEV = "cuda"
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")

# (rank 0 items, rank 1 items) per step; item i is window i % 2 of the dataset
STEPS = [([0, 2, 4], [6, 8]),          # one window on both ranks (comparable with the union batch)
         ([10, 1, 3], [5])]            # rank 0: two window groups, rank 1: one


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup():
    from src.dataset.synthetic import make_rag_dataset
    from src.model import build_model
    torch.manual_seed(0)
    np.random.seed(0)                   # the construction-time window masks draw from the global RNG
    ds, vocab = make_rag_dataset(n_samples=8, n_sites=300, n_windows=2, n_ref_samples=40, seed=5, name="train")
    ds.panel_cache = "fresh"
    m = build_model(len(vocab), 128, 2, 4, dropout=0.0).to(DEV)
    for mod in m.modules():                     # incl. the reference's fixed 0.1 dropouts (fusion.py)
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    return ds, vocab, m


def _trainer(m, ds, vocab, bucket_bytes=256 << 10):
    from src.main.pretrain_with_val_optimized import BERTTrainerWithValidationOptimized
    tr = BERTTrainerWithValidationOptimized(m, None, None, vocab, lr=1e-3, warmup_steps=1, grad_accum_steps=1,
                                            log_freq=0, bucket_bytes=bucket_bytes)
    tr.rag_train_dataset = ds
    tr.rag_k = 4
    captured = []
    orig = tr.optim.step

    def step(grad_scale=1.0):           # the reduced gradient and the weights the step starts from
        captured.append((tr.flat.grad.detach().cpu().clone(), tr.flat.flat.detach().cpu().clone(), grad_scale))
        orig(grad_scale)
        torch.cuda.synchronize()
        post.append(dict(flat=tr.flat.flat.detach().cpu().clone(), sq=float(tr.optim.sq.item()),
                         lr=float(tr.optim.param_groups[0]["lr"]), step=tr.optim.step_count))
    post = []
    tr.optim.step = step
    tr._post = post
    return tr, captured


def _batch(ds, items):
    from src.dataset.embedding_rag_dataset import embedding_rag_collate_fn
    return embedding_rag_collate_fn([ds[i] for i in items])


def _ddp_worker(rank, world, port, panel, q):
    import faulthandler
    faulthandler.dump_traceback_later(170, exit=True)
    sys.path[:0] = [ROOT, os.path.join(ROOT, "rag-snvbert_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from src.retrieval.shards import PanelShard
        ds, vocab, m = _setup()
        if panel == "sharded":
            ds.set_panel_shard(PanelShard.current())
        final_at, trace = {}, []
        for p in m.parameters():        # registered before the bucketer's own hooks: they run first
            p.register_post_accumulate_grad_hook(lambda _p, k=id(p): final_at.update({k: len(trace)}) and None)
        tr, captured = _trainer(m, ds, vocab)
        bk = tr.ddp
        assert bk.active and len(bk.buckets) >= 8, len(bk.buckets)
        bk.trace = trace
        checks = []
        for items in STEPS:
            final_at.clear()
            trace.clear()
            tr.train_step(_batch(ds, items[rank]))
            order = [b for b, _ in trace]
            fin = lambda i: final_at.get(id(tr.flat.params[i]))
            # launched with exactly the members that were final; the others got no gradient at all
            # this step (launched by finish())
            complete = all(ready == frozenset(i for i in bk.buckets[b] if fin(i) is not None) for b, ready in trace)
            # a member became final at or before the launch position of its bucket
            early = [(b, i) for t, (b, _) in enumerate(trace) for i in bk.buckets[b]
                     if fin(i) is not None and fin(i) > t]
            unused = sorted(i for b, _ in trace for i in bk.buckets[b] if fin(i) is None)
            # buckets launched from the post-accumulate hooks during backward (every member final),
            # as opposed to by finish() after it
            hooked = sum(1 for b, ready in trace if len(ready) == len(bk.buckets[b]))
            checks.append(dict(order=order, complete=complete, early=early, n_final=len(final_at),
                               unused=unused, hooked=hooked))
        names = {id(p): n for n, p in m.named_parameters()}
        q.put((rank, dict(checks=checks, steps=[(g.numpy(), f.numpy(), s) for g, f, s in captured],
                          post=[dict(d, flat=d["flat"].numpy()) for d in tr._post],
                          final=tr.flat.flat.detach().cpu().numpy(), n_buckets=len(bk.buckets),
                          buckets=[list(b) for b in bk.buckets],
                          names=[names[id(p)] for p in tr.flat.params], offsets=list(tr.flat.offsets))))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _spawn(target, args_fn, n=2, timeout=280):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=target, args=(r, n, port) + args_fn(r) + (q,)) for r in range(n)]
    for p in ps:
        p.start()
    try:
        got = dict(q.get(timeout=timeout) for _ in ps)
    finally:
        for p in ps:
            p.join(30)
            if p.is_alive():
                p.kill()
                p.join(10)
    for r, v in got.items():
        assert not isinstance(v, str), f"rank {r}:\n{v}"
    for p in ps:
        assert p.exitcode == 0
    return got


def _replay_grad(flat_before, items):
    """Single process (world 1): the gradient of one batch from the given weights."""
    ds, vocab, m = _setup()
    tr, captured = _trainer(m, ds, vocab)
    tr.flat.flat.copy_(torch.from_numpy(flat_before).to(DEV))
    tr.flat.sync_mirror()
    tr.train_step(_batch(ds, items))
    return captured[0][0].numpy()


def _adam_host(p, g, sq, lr, step, scale, b1=0.9, b2=0.999, eps=1e-8, wd=0.01, max_norm=1.0):
    """FusedAdam's first step (m = v = 0) in float64 from the captured inputs."""
    p, g = p.astype(np.float64), g.astype(np.float64)
    coef = scale * min(max_norm / (np.sqrt(sq) * scale + 1e-6), 1.0)
    gi = g * coef + wd * p
    m, v = (1 - b1) * gi, (1 - b2) * gi * gi
    return p - lr / (1 - b1 ** step) * m / (np.sqrt(v) / np.sqrt(1 - b2 ** step) + eps)


def _rel(a, b):
    return float(np.linalg.norm(a.astype(np.float64) - b) / max(np.linalg.norm(b.astype(np.float64)), 1e-30))


@pytest.mark.timeout(600)
@pytest.mark.parametrize("panel", ["sharded", "replicated"])
def test_ddp_train_step_buckets_final_and_ranks_equal(panel):
    got = _spawn(_ddp_worker, lambda r: (panel,))
    r0, r1 = got[0], got[1]
    for s in range(len(STEPS)):
        for r in (0, 1):
            c = got[r]["checks"][s]
            assert c["order"] == list(range(got[r]["n_buckets"])), (r, s, c["order"])
            assert c["complete"] and not c["early"], (r, s, c)
            assert c["unused"] == got[0]["checks"][0]["unused"] and c["n_final"] > 50, (r, s, c)
            # every parameter in the graph reports through its hook — Linear / LayerNorm weights
            # under direct_weight_grads included — so all buckets but those holding a parameter
            # with no gradient this step (and the ones after it) launch during backward
            # (rag_fusion.pooling: its softmax runs over ONE neighbour mean, train_forward.py:137,
            # so its weight is exactly 1 and its Linear gets no gradient — zero in the reference)
            unused_names = [got[r]["names"][i] for i in c["unused"]]
            assert all(".pooling." in n for n in unused_names), (r, s, unused_names)
            first_unused = min((b for b, members in enumerate(got[r]["buckets"]) if set(members) & set(c["unused"])),
                               default=got[r]["n_buckets"])
            assert c["hooked"] >= first_unused, (r, s, c["hooked"], first_unused, unused_names)
        g0, f0, sc0 = r0["steps"][s]
        g1, f1, sc1 = r1["steps"][s]
        assert sc0 == sc1 == 1.0
        # identical weights going into the step and identical reduced gradients on both ranks
        df, dg = np.nonzero(f0 != f1)[0], np.nonzero(g0 != g1)[0]
        for r in (0, 1) if s == 0 else ():   # the first Adam step consumed the reduced gradient
            pr, (gr, fr, sc) = got[r]["post"][s], got[r]["steps"][s]
            d = np.abs(pr["flat"] - _adam_host(fr, gr, pr["sq"], pr["lr"], pr["step"], sc))
            assert d.max() <= 1e-5, (panel, r, float(d.max()))
        where = lambda ix: sorted({got[0]["names"][int(np.searchsorted(got[0]["offsets"], i, "right")) - 1]
                                   for i in ix[:2000]})[:12]
        assert df.size == 0 and dg.size == 0, (panel, s, df.size, dg.size, where(df), where(dg),
                                               float(np.abs(g0 - g1).max()))
        # the reduced gradient == the sum of the two ranks' single-process gradients
        want = _replay_grad(f0, STEPS[s][0]).astype(np.float64) + _replay_grad(f0, STEPS[s][1])
        rel = _rel(g0, want)
        print(f"{panel} step {s}: reduced vs sum of per-rank single-process gradients rel {rel:.2e}")
        assert rel <= 1e-5, rel
        if s == 0:
            # one window on both ranks: the same BatchNorm batch statistics as the union batch
            union = _replay_grad(f0, STEPS[0][0] + STEPS[0][1])
            rel_u = _rel(g0, union)
            print(f"{panel} step 0: reduced vs single-process union-batch gradient rel {rel_u:.2e}")
            assert rel_u <= 1e-3, rel_u
    np.testing.assert_array_equal(r0["final"], r1["final"])


# ------------------------------------------------------------------ entry point, 2 ranks --
_MAIN_ARGS = ["--synthetic", "8", "--synthetic_sites", "300", "--synthetic_windows", "1", "--synthetic_ref", "40",
              "--dims", "128", "--layers", "2", "--attn_heads", "4", "--epochs", "3", "--patience", "1",
              "--lr", "0", "--dropout", "0", "--grad_accum_steps", "1", "--rag_k", "4", "--log_freq", "0",
              "--warmup_steps", "1"]


def _record_samples(rec):
    """Per train / val sample (keyed by its token and mask bytes): the retrieved neighbours of both
    haplotypes and the sample's three focal-loss parts — so a mismatch of the epoch rows below
    names the samples and says whether retrieval or the forward moved (tools/ddp_diag.py)."""
    import hashlib
    from src.main import pretrain_with_val_optimized as T
    cls = T.BERTTrainerWithValidationOptimized
    orig_epoch, orig_loss, state = cls._run_epoch, cls.loss, {}

    def run_epoch(self, epoch, dataloader, train=True):
        state.update(epoch=epoch, train=train)
        return orig_epoch(self, epoch, dataloader, train)

    def loss(self, output, data):
        r = orig_loss(self, output, data)
        with torch.no_grad():
            m = data["mask"].bool()
            for i in range(m.shape[0]):
                key = hashlib.sha1(b"".join(data[k][i].cpu().numpy().tobytes() for k in ("hap_1", "hap_2", "mask")))
                parts = [float(self.hap_criterion(output[j][i:i + 1], data[lab][i:i + 1], m[i:i + 1]))
                         for j, lab in ((0, "hap_1_label"), (1, "hap_2_label"))]
                parts.append(float(self.gt_criterion(output[2][i:i + 1], data["gt_label"][i:i + 1], m[i:i + 1])))
                idx = [data[k][i].cpu().tolist() if k in data else None for k in ("rag_idx_h1", "rag_idx_h2")]
                rec[(state["epoch"], state["train"], key.hexdigest()[:16])] = (idx, parts)
        return r
    cls._run_epoch, cls.loss = run_epoch, loss
    return lambda: setattr(cls, "_run_epoch", orig_epoch) or setattr(cls, "loss", orig_loss)


def _main_worker(rank, world, port, out, q):
    import faulthandler
    faulthandler.dump_traceback_later(250, exit=True)
    sys.path[:0] = [ROOT, os.path.join(ROOT, "rag-snvbert_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK="0")
    try:
        from src import train_embedding_rag
        rec = {}
        _record_samples(rec)
        tr = train_embedding_rag.main(_MAIN_ARGS + ["--train_batch_size", "2", "--val_batch_size", "1",
                                                    "--dist_backend", "gloo", "--panel", "sharded",
                                                    "--metrics_csv", os.path.join(out, "m.csv"),
                                                    "--output_path", os.path.join(out, f"r{rank}", "model")])
        q.put((rank, dict(epochs=len(tr.epoch_metrics), best=tr.best_val_metric, no_imp=tr.epochs_no_improve,
                          bn=[b.detach().cpu().numpy() for b in tr.model.buffers()], samples=rec)))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


@pytest.mark.timeout(600)
def test_train_main_two_ranks_global_metrics_and_early_stop(tmp_path):
    """lr 0 and dropout 0: the weights stay at their (broadcast) initial values and the BatchNorm
    batch statistics of a one-window dataset are the same for every batch, so the two-rank run
    (per-rank batch 2 / 1) and one process with the global batch (4 / 2) see the same function on
    the same samples — their epoch CSV rows must agree: F1 / precision / recall / accuracy
    exactly (summed integer counts), the loss to float rounding."""
    got = _spawn(_main_worker, lambda r: (str(tmp_path),), timeout=500)
    assert got[0]["epochs"] == got[1]["epochs"] and got[0]["no_imp"] == got[1]["no_imp"]
    assert got[0]["best"] == got[1]["best"]
    for a, b in zip(got[0]["bn"], got[1]["bn"]):
        np.testing.assert_array_equal(a, b)
    ddp = _rows(tmp_path / "m.csv")
    assert len(ddp) == got[0]["epochs"] and got[0]["epochs"] < 2 * 3   # stopped early (patience 1)
    from src import train_embedding_rag
    single = tmp_path / "single"
    one = {}
    restore = _record_samples(one)
    try:
        tr = train_embedding_rag.main(_MAIN_ARGS + ["--train_batch_size", "4", "--val_batch_size", "2",
                                                    "--metrics_csv", str(single / "m.csv"),
                                                    "--output_path", str(single / "model")])
    finally:
        restore()
    # per sample first: the same neighbours and the same loss parts as the one-process run
    two = {**got[0]["samples"], **got[1]["samples"]}
    assert sorted(two) == sorted(one), (len(two), len(one))
    bad = [(k, two[k], one[k]) for k in sorted(one)
           if two[k][0] != one[k][0] or not np.allclose(two[k][1], one[k][1], rtol=1e-5, atol=1e-6)]
    assert not bad, f"{len(bad)} samples differ (epoch, train, key): (two-rank idx, parts) vs one process: {bad[:4]}"
    ref = _rows(single / "m.csv")
    assert len(ref) == len(ddp) and len(tr.epoch_metrics) == got[0]["epochs"]
    for a, b in zip(ddp, ref):
        assert (a["epoch"], a["mode"]) == (b["epoch"], b["mode"])
        for k in a:
            if k in ("epoch", "mode"):
                continue
            if k == "loss":
                np.testing.assert_allclose(float(a[k]), float(b[k]), rtol=1e-5)
            else:
                assert float(a[k]) == float(b[k]), (k, a, b)
