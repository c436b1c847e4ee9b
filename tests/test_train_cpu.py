"""CPU tests of the training path: the oracle against the reference's own autograd values
(tests/golden/focal.npz, train_tiny.npz), the LR schedule, and the data-parallel gradient
bucketing over a world-size-2 gloo group (the same code runs over RCCL on the GPUs)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_golden
from oracle import train_np


def test_focal_oracle_matches_reference_autograd():
    z = load_golden("focal")
    for C in (2, 4):
        loss, grad = train_np.focal_loss(z[f"x{C}"], z[f"y{C}"], z[f"m{C}"], 2.0)
        np.testing.assert_allclose(loss, float(z[f"loss{C}"]), rtol=1e-5)
        np.testing.assert_allclose(grad, z[f"grad{C}"], rtol=1e-4, atol=1e-7)


def test_focal_oracle_on_model_outputs():
    """The train_tiny loss values re-derived from the reference's own output probabilities."""
    g = load_golden("train_tiny")
    m = g["mask"].astype(bool)
    l1, _ = train_np.focal_loss(g["probs_h1"].reshape(-1, 2), g["hap_1_label"].reshape(-1), m.reshape(-1))
    lg, _ = train_np.focal_loss(g["gt"].reshape(-1, 4), g["gt_label"].reshape(-1), m.reshape(-1))
    np.testing.assert_allclose([l1, lg], g["losses"][[0, 2]], rtol=1e-5)


def test_scheduled_optim_matches_reference_formula():
    from src.main.optim_schedule import ScheduledOptim

    class _Opt:
        param_groups = [{"lr": 0.0}]
    s = ScheduledOptim(_Opt(), n_warmup_steps=10, init_lr=1e-5, max_lr=5e-5)
    for step in range(1, 30):
        s.step()
        assert abs(_Opt.param_groups[0]["lr"] - train_np.lr_schedule(step, 10, 1e-5, 5e-5)) < 1e-15


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _index(fp, p):
    return next(i for i, t in enumerate(fp.params) if t is p)


def _bucket_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from src.main.optimizer import FlatParams, GradBucketer
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 8),
                                  torch.nn.Linear(8, 4))
        unused = torch.nn.Linear(3, 3)       # no gradient this step: its bucket still reduces
        ref = [p.detach().clone() for p in net.parameters()]
        fp = FlatParams(list(net.parameters()) + list(unused.parameters()), mirror=False)
        bk = GradBucketer(fp, bucket_bytes=600)
        assert len(bk.buckets) >= 3
        x = torch.randn(5, 16, generator=torch.Generator().manual_seed(rank))
        for micro in range(2):             # grad accumulation: sync on the second micro-step only
            bk.enabled = micro == 1
            net(x * (micro + 1)).pow(2).sum().backward()
        scale = bk.finish()
        assert scale == 1.0
        avg = (fp.grad * scale).clone()
        # expected: SUM over ranks of the locally accumulated gradients (the reference's
        # DataParallel gradient of one summed loss over the global batch)
        local = []
        for r in range(world):
            n2 = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 8),
                                     torch.nn.Linear(8, 4))
            with torch.no_grad():
                for p, v in zip(n2.parameters(), ref):
                    p.copy_(v)
            xr = torch.randn(5, 16, generator=torch.Generator().manual_seed(r))
            for micro in range(2):
                n2(xr * (micro + 1)).pow(2).sum().backward()
            local.append([p.grad.clone() for p in n2.parameters()])
        ok = True
        for i, p in enumerate(net.parameters()):
            exp = sum(l[i] for l in local)
            got = fp.view(avg, _index(fp, p))
            ok &= torch.allclose(got, exp, rtol=1e-5, atol=1e-6)
        for p in unused.parameters():
            ok &= bool((fp.view(avg, _index(fp, p)) == 0).all())
        q.put((rank, bool(ok)))
    except Exception as e:          # report instead of leaving the parent waiting
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_grad_bucketer_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=200) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {r: True for r in range(world)}


class _DirectLinear(torch.autograd.Function):
    """A Linear whose backward adds dW / db straight into ``w.grad`` / ``b.grad`` and returns None
    for them — the shape of autograd_ops' HIP Linear under direct_weight_grads."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w, b)
        return x @ w.t() + b

    @staticmethod
    def backward(ctx, gy):
        x, w, b = ctx.saved_tensors
        w.grad.add_(gy.t() @ x)
        b.grad.add_(gy.sum(0))
        return gy @ w, None, None


def _shared_use_worker(rank, world, port, q):
    """A graph where the first-registered parameters (the LAST bucket, as the AF MLP is) are used
    a rank-dependent number of times through the direct-accumulation path plus once through
    autograd: every bucket must launch only after all of its parameters are final, in the same
    order on both ranks, and the reduced gradient must equal the sum of the ranks' full
    gradients."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from src.main.optimizer import FlatParams, GradBucketer
        torch.manual_seed(0)
        shared = torch.nn.Linear(8, 8)                 # registered first -> last bucket
        body = torch.nn.Linear(8, 8)
        head = torch.nn.Linear(8, 2)
        params = list(shared.parameters()) + list(body.parameters()) + list(head.parameters())
        init = [p.detach().clone() for p in params]
        fp = FlatParams(params, mirror=False)
        trace = []
        final_at = {}               # param index -> launches issued when it became final
        for i, p in enumerate(fp.params):           # registered before the bucketer's hooks: run first
            p.register_post_accumulate_grad_hook(lambda _p, i=i: final_at.update({i: len(trace)}) and None)
        bk = GradBucketer(fp, bucket_bytes=300)
        assert len(bk.buckets) >= 3
        bk.trace = trace

        def fwd(x, n_uses, direct):
            lin = (lambda t, m: _DirectLinear.apply(t, m.weight, m.bias)) if direct else (lambda t, m: m(t))
            h = sum(lin(x * (u + 1), shared) for u in range(n_uses))   # rank-dependent use count
            h = torch.tanh(lin(h, body))
            return shared(torch.tanh(head(h)).repeat(1, 4)).pow(2).sum()   # one autograd use too

        n_uses = _uses(rank)
        x = torch.randn(5, 8, generator=torch.Generator().manual_seed(rank))
        fwd(x, n_uses, True).backward()
        assert bk.finish() == 1.0
        order = [b for b, _ in bk.trace]
        ok = order == list(range(len(bk.buckets)))
        ok &= all(ready == frozenset(bk.buckets[b]) for b, ready in bk.trace)
        # no bucket launched before one of its members was final
        ok &= all(final_at[i] <= b for b, _ in bk.trace for i in bk.buckets[b])
        # expected: sum over ranks of plain-autograd gradients
        exp = torch.zeros_like(fp.grad)
        for r in range(world):
            ps = [torch.nn.Parameter(t.clone()) for t in init]
            s2, b2, h2 = torch.nn.Linear(8, 8), torch.nn.Linear(8, 8), torch.nn.Linear(8, 2)
            for m, (w, b) in zip((s2, b2, h2), zip(ps[0::2], ps[1::2])):
                m.weight, m.bias = w, b
            xr = torch.randn(5, 8, generator=torch.Generator().manual_seed(r))
            shared_, body_, head_ = s2, b2, h2
            h = sum(shared_(xr * (u + 1)) for u in range(_uses(r)))
            h = torch.tanh(body_(h))
            shared_(torch.tanh(head_(h)).repeat(1, 4)).pow(2).sum().backward()
            for j, p in enumerate(ps):
                fp.view(exp, _index_of(fp, params[j])).add_(p.grad)
        ok &= torch.allclose(fp.grad, exp, rtol=1e-5, atol=1e-6)
        q.put((rank, (bool(ok), order)))
    except Exception as e:
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _index_of(fp, p):
    return next(i for i, t in enumerate(fp.params) if t is p)


def _uses(rank):
    """Rank-dependent use count of the shared layer (1..4): its bucket finishes at a different
    point of every rank's backward."""
    return (3, 1, 4, 2, 1, 3, 2, 4)[rank % 8]


@pytest.mark.parametrize("world", [2, 8])
def test_grad_bucketer_launches_after_last_use_in_rank_order(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shared_use_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=200) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(res[r] == res[0] for r in range(world)) and res[0][0] is True, res


def test_trainer_metric_rows_and_early_stopping_match_reference(tmp_path):
    """The trainer's per-epoch CSV rows (ALT-class F1 / precision / recall overall, rare and
    common; loss; accuracy — pretrain_with_val_optimized.py:424-488) and its early-stopping
    decisions on hap_f1[1] (:490-522), with the `is_best` flag taken before the update
    (train_embedding_rag.py:405-409), equal the reference's on the same counts
    (tests/golden/metrics.npz, generated by running the reference's methods)."""
    import csv
    from types import SimpleNamespace
    from src.main.pretrain_with_val_optimized import BERTTrainerWithValidationOptimized as T
    z = load_golden("metrics")
    n = len(z["stops"])
    st = SimpleNamespace(calculate_metrics=T.calculate_metrics, best_val_metric=-np.inf, min_delta=0.001,
                         epochs_no_improve=0, patience=2, val_metric="f1", rank=1,
                         output_csv=str(tmp_path / "m.csv"))
    stops, bests = [], []
    for e in range(n):
        g = lambda k: torch.from_numpy(z[f"{e}:{k}"])
        counts = {name: torch.stack([g(f"{name}_tp"), g(f"{name}_fp"), g(f"{name}_fn")])
                  for name in ("hap", "rare", "common")}
        row = T.metric_row(st, e, e % 2 == 0, counts, float(z[f"{e}:hap_loss"]), int(z["num_batches"][e]),
                           int(z[f"{e}:hap_correct"]), int(z[f"{e}:hap_numbers"]))
        T._save_epoch_metrics(st, row)
        bests.append(st.epochs_no_improve == 0)
        stops.append(T.should_stop_early(st, {f"hap_{k}": g(f"hap_{k}") for k in ("tp", "fp", "fn")}, e))
    with open(st.output_csv) as f:
        rows = list(csv.reader(f))
    assert rows[0] == list(z["header"])
    np.testing.assert_array_equal(np.array(rows[1:]), z["rows"])
    assert stops == list(z["stops"]) and bests == list(z["is_best_before"])


def test_pos_feat_batchnorm_matches_module_with_repeated_updates():
    """train_forward._batchnorm (the pos_feat BatchNorms in torch ops) == nn.BatchNorm1d in
    train mode: output, input / affine gradients (f64), and the running statistics after n
    reference calls on the same batch; eval mode uses the running statistics."""
    import copy
    from src.train_forward import _batchnorm
    torch.manual_seed(0)
    bn = torch.nn.BatchNorm1d(4).double()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    ref = copy.deepcopy(bn)
    x = (torch.randn(2, 4, 1030, dtype=torch.float64) * 3 + 1).requires_grad_(True)
    xr = x.detach().clone().requires_grad_(True)
    g = torch.randn(2, 4, 1030, dtype=torch.float64)
    y = _batchnorm(bn, x, n_updates=4)
    yr = ref(xr)
    for _ in range(3):
        with torch.no_grad():
            ref(xr)
    torch.testing.assert_close(y, yr, rtol=1e-12, atol=1e-12)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-10, atol=1e-12)
    torch.testing.assert_close(bn.weight.grad, ref.weight.grad, rtol=1e-10, atol=1e-12)
    torch.testing.assert_close(bn.bias.grad, ref.bias.grad, rtol=1e-10, atol=1e-12)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, rtol=1e-12, atol=1e-14)
    torch.testing.assert_close(bn.running_var, ref.running_var, rtol=1e-12, atol=1e-14)
    assert int(bn.num_batches_tracked) == int(ref.num_batches_tracked) == 4
    bn.eval()
    ref.eval()
    torch.testing.assert_close(_batchnorm(bn, x.detach()), ref(x.detach()), rtol=1e-12, atol=1e-12)


def test_grad_sketch_estimator_on_reference_gradients():
    """tests/grad_sketch.py (the v18 fixture's gradient storage): on the train_tiny reference
    gradients a sketch compares exactly to its own gradient, and a perturbation of relative size
    1e-2 is estimated within a factor 2; the committed train_v18 sketch is consistent (norms
    positive, 16 projections per parameter)."""
    import grad_sketch as GS
    g = load_golden("train_tiny")
    rng = np.random.default_rng(0)
    ratios = []
    for key in (k for k in g if k.startswith("g:")):
        name, r = key[2:], g[key]
        if np.linalg.norm(r) == 0:
            continue
        sk = GS.sketch(name, r)
        est, rel_s, cos = GS.compare(name, r, sk)
        assert est == 0 and rel_s == 0 and abs(cos - 1) < 1e-6
        e = rng.standard_normal(r.shape).astype(np.float32)
        e *= 1e-2 * np.linalg.norm(r) / np.linalg.norm(e)
        ratios.append(GS.compare(name, r + e, sk)[0] / 1e-2)
    assert 0.6 < np.median(ratios) < 1.4 and min(ratios) > 0.3 and max(ratios) < 2.2, ratios
    v = load_golden("train_v18")
    names = GS.names(v)
    assert len(names) > 250 and all(v[f"gp:{n}"].shape == (GS.NPROJ,) for n in names)


def _torch_focal(p, y, m, gamma=2.0):
    """FocalLoss(gamma, 'sum') on probability rows (optim_schedule.py:49-96), torch f64."""
    p, y, m = p.reshape(-1, p.shape[-1]).double(), y.reshape(-1), m.reshape(-1)
    pt = p.gather(1, y[:, None])[:, 0].clamp(min=1e-12)
    return (-(1 - pt) ** gamma * pt.log())[m].sum()


@pytest.mark.parametrize("scale", [1.0, 1e-3])
def test_recon_loss_branch_matches_reference_formula(scale):
    """use_recon_loss=True (pretrain_with_val_optimized.py:219-228): nn.MSELoss between outputs 3/5
    and 4/6 at the masked sites; both above MIN_RECON_LOSS -> 0.2 FL1 + 0.2 FL2 + 0.3 FLgt + 0.15
    MSE1 + 0.15 MSE2, else 3 FL1 + 3 FL2 + 4 FLgt; / grad_accum_steps.  ``scale`` 1e-3 puts the MSEs
    below the threshold; the gradient flows into the raw and encoded embeddings."""
    from types import SimpleNamespace
    from src.main.pretrain_with_val_optimized import BERTTrainerWithValidationOptimized as T, MIN_RECON_LOSS
    g = torch.Generator().manual_seed(1)
    B, L, D = 2, 30, 8
    sm = lambda *s: torch.softmax(torch.randn(*s, generator=g), -1)
    out = [sm(B, L, 2), sm(B, L, 2), sm(B, L, 4)] + \
          [(scale * torch.randn(B, L, D, generator=g)).requires_grad_(True) for _ in range(4)]
    data = {"mask": (torch.rand(B, L, generator=g) < 0.4).long(),
            "hap_1_label": torch.randint(0, 2, (B, L), generator=g), "hap_2_label": torch.randint(0, 2, (B, L), generator=g),
            "gt_label": torch.randint(0, 4, (B, L), generator=g)}
    crit = lambda p, y, m: _torch_focal(p, y, m).float()
    st = SimpleNamespace(grad_accum_steps=2, use_recon_loss=True, hap_criterion=crit, gt_criterion=crit)
    total, (l1, l2, lg) = T.loss(st, out, data)
    m = data["mask"].bool()
    mse = torch.nn.MSELoss()
    r1, r2 = mse(out[3][m], out[5][m]), mse(out[4][m], out[6][m])
    if r1 > MIN_RECON_LOSS and r2 > MIN_RECON_LOSS:
        want = 0.2 * l1 + 0.2 * l2 + 0.3 * lg + 0.15 * r1 + 0.15 * r2
    else:
        want = 3 * l1 + 3 * l2 + 4 * lg
    assert (scale == 1.0) == bool(r1 > MIN_RECON_LOSS)
    torch.testing.assert_close(total, want / 2, rtol=1e-5, atol=1e-6)
    total.backward()
    gr = out[3].grad
    if scale == 1.0:
        assert gr is not None and gr.abs().sum() > 0
    else:
        assert gr is None or float(gr.abs().sum()) == 0.0
    st.use_recon_loss = False
    total2, _ = T.loss(st, out, data)
    torch.testing.assert_close(total2, (3 * l1 + 3 * l2 + 4 * lg) / 2)


class _StubModel(torch.nn.Module):
    """Outputs a fixed function of the batch (probabilities from the tokens), so two ranks and one
    process see the same per-sample outputs."""

    def __init__(self):
        super().__init__()
        self.w = torch.nn.Parameter(torch.zeros(1))
        self.bert = torch.nn.Module()
        self.bert.embedding = torch.nn.Module()          # the trainer's retrieval handle (unused here)

    def forward(self, x):
        h = x["hap_1"].double()
        p1 = torch.sigmoid(torch.sin(h * 1.7 + x["af"].double()))
        p2 = torch.sigmoid(torch.cos(h * 0.9))
        pg = torch.softmax(torch.stack([h.sin(), h.cos(), (2 * h).sin(), x["af"].double()], -1), -1)
        two = lambda p: torch.stack([1 - p, p], -1).float()
        return [two(p1), two(p2), pg.float()]


def _stub_batches(items):
    g = torch.Generator().manual_seed(7)
    L = 40
    tok = torch.randint(4, 7, (16, L), generator=g)
    af = torch.rand(16, L, generator=g)
    mask = (torch.rand(16, L, generator=g) < 0.5).long()
    lab = torch.randint(0, 2, (16, L), generator=g)
    gl = torch.randint(0, 4, (16, L), generator=g)
    out = []
    for b in items:
        i = torch.tensor(b)
        out.append({"hap_1": tok[i], "af": af[i], "mask": mask[i], "hap_1_label": lab[i], "hap_2_label": 1 - lab[i],
                    "gt_label": gl[i]})
    return out


def _patch_trainer_cpu(T, tr):
    """CPU stand-ins for the two HIP kernels the epoch loop calls (focal loss, confusion counts)."""
    from src.main import optim_schedule as OS
    crit = lambda p, y, m: _torch_focal(p, y, m).float()
    tr.hap_criterion = tr.gt_criterion = crit

    def upd(self, probs, labels, mask, mask2=None):
        m = mask.bool() if mask2 is None else (mask.bool() & mask2.bool())
        c = train_np.confusion(probs.detach().numpy(), labels.numpy(), m.numpy(), self.C)
        self.counts += torch.from_numpy(c)
    OS.DeviceConfusion.update = upd


def _metric_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from src.main.pretrain_with_val_optimized import BERTTrainerWithValidationOptimized as T
        m = _StubModel()
        tr = T(m, None, _stub_batches([[0, 1, 2], [3, 4]] if rank == 0 else [[5, 6, 7], [8, 9]]), None,
               log_freq=0, patience=1)
        _patch_trainer_cpu(T, tr)
        res = tr.validate(0)
        stop1 = tr.should_stop_early(res, 0)
        stop2 = tr.should_stop_early(res, 1)
        q.put((rank, ({k: v for k, v in res.items() if not torch.is_tensor(v) and k != "sec"},
                      {k: v.tolist() for k, v in res.items() if torch.is_tensor(v)}, stop1, stop2)))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_epoch_metrics_summed_over_ranks_gloo_world2():
    """The trainer's epoch metrics under two gloo ranks (pretrain_with_val_optimized.py:362-372,
    :490-522): losses and TP/FP/FN summed over ranks, the batch count = global steps, the CSV row
    and the early-stopping decision identical on both ranks and equal to one process that ran the
    union of the samples with the global batch (rank batches 3 + 3 and 2 + 2)."""
    from src.main.pretrain_with_val_optimized import BERTTrainerWithValidationOptimized as T
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_metric_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert not isinstance(got[0], str), got[0]
    assert not isinstance(got[1], str), got[1]
    assert got[0] == got[1]
    from src.main import optim_schedule as OS
    orig = OS.DeviceConfusion.update
    try:
        tr = T(_StubModel(), None, _stub_batches([[0, 1, 2, 5, 6, 7], [3, 4, 8, 9]]), None, log_freq=0, patience=1)
        _patch_trainer_cpu(T, tr)
        res = tr.validate(0)
    finally:
        OS.DeviceConfusion.update = orig
    row, counts, s1, s2 = got[0]
    assert row["batches"] == res["batches"] == 2
    for k, v in row.items():
        if isinstance(v, float):
            np.testing.assert_allclose(v, res[k], rtol=1e-5, err_msg=k)
        else:
            assert v == res[k], k
    for k, v in counts.items():
        assert v == res[k].tolist(), k
    assert (s1, s2) == (False, True)
