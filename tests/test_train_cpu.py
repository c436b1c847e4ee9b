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
        avg = (fp.grad * scale).clone()
        # expected: mean over ranks of the locally accumulated gradients
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
            exp = sum(l[i] for l in local) / world
            got = fp.view(avg, _index(fp, p))
            ok &= torch.allclose(got, exp, rtol=1e-5, atol=1e-6)
        for p in unused.parameters():
            ok &= bool((fp.view(avg, _index(fp, p)) == 0).all())
        q.put((rank, bool(ok)))
    except Exception as e:          # report instead of leaving the parent waiting
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_grad_bucketer_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


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
