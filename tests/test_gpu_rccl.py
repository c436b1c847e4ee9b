"""The RCCL ("nccl" backend) code paths of the multi-GPU design, executed once on the one GPU
of the test box: a world-size-1 nccl process group in a spawned child process runs exactly the
collectives the 8-GPU path issues (src/retrieval/shards.py, src/main/optimizer.py):

  * ``_all_gather`` -> ``all_gather_into_tensor`` on u8 (query tokens) and int64 (top-k keys);
  * ``all_gather_rows`` (the ragged-count exchange + padded gather);
  * the u8 SUM ``all_reduce`` of the neighbours' alt-allele counts (``_all_reduce``);
  * ``sharded_neighbours`` over the HIP kernels (eval counts form, and the train-mode form with
    dropped-out query offsets and the unique neighbours' code exchange) == the single-index search;
  * one ``GradBucketer`` step whose buckets are all-reduced asynchronously over RCCL.

With one rank each collective is an identity, so the results are checked exactly; what the test
proves is that the dtypes, shapes and call forms are accepted and run by RCCL on gfx950.
Scaling across ranks is not measured here."""

import os
import socket
import traceback

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(port, q):
    import faulthandler
    import sys
    faulthandler.dump_traceback_later(80, exit=True)   # a hung collective names itself, then exits
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
    sys.path[:0] = [root, os.path.join(root, "rag-snvbert_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        from src.retrieval import shards
        from src.retrieval import PanelIndex
        from src import kernels as K
        from src.main.optimizer import FlatParams, GradBucketer
        done = []
        print("nccl up", flush=True)
        x8 = torch.arange(4 * 70, device=dev, dtype=torch.int64).remainder(251).to(torch.uint8).view(4, 70)
        g8 = shards._all_gather(x8)
        assert g8.shape == (1, 4, 70) and g8.dtype == torch.uint8 and torch.equal(g8[0], x8)
        x64 = torch.randint(-2 ** 62, 2 ** 62, (5, 8), device=dev, dtype=torch.int64)
        g64 = shards._all_gather(x64)
        assert torch.equal(g64[0], x64)
        done.append("all_gather_into_tensor u8/int64")
        print(done[-1], flush=True)
        rows, sizes = shards.all_gather_rows(torch.randn(3, 7, device=dev))
        assert sizes == [3] and rows.shape == (3, 7)
        done.append("all_gather_rows")
        print(done[-1], flush=True)
        c = shards._all_reduce(x8.clone(), dist.ReduceOp.SUM)
        assert torch.equal(c, x8)
        assert shards.any_rank(True, dev) and not shards.any_rank(False, dev)
        done.append("all_reduce u8 SUM / int32 MAX")
        print(done[-1], flush=True)
        # the sharded search on the HIP kernels, a world of one == the plain index search
        rng = np.random.default_rng(1)
        N, S, L, D, k = 3000, 300, 1030, 64, 8
        af = torch.from_numpy(rng.beta(0.3, 3.0, S).astype(np.float32)).to(dev)
        codes = K.panel_synth(N, S, af, 5)
        index = PanelIndex(codes, S, torch.zeros(L, device=dev))
        W = torch.from_numpy(rng.standard_normal((12, D)).astype(np.float32)).to(dev)
        site_mask = torch.from_numpy((rng.random(S) < 0.4).astype(np.uint8)).to(dev)
        tok = torch.zeros(9, L, dtype=torch.long, device=dev)
        tok[:, 0], tok[:, S + 1] = 2, 3
        qr = codes[torch.from_numpy(rng.integers(0, N, 9)).to(dev), :S].long()
        tok[:, 1:S + 1] = torch.where(site_mask.bool()[None], torch.full_like(qr, 4), 5 + qr)
        ops = shards.kernel_ops(index, W, site_mask, k)
        idx, _, counts = shards.sharded_neighbours(tok, k, ops)
        want, _ = index.search(tok, W, site_mask, k)
        assert torch.equal(idx, want)
        assert torch.equal(counts, K.neighbor_counts(want, codes, 0))
        # train-mode form: per-query offsets travel with the tokens, codes of the unique neighbours
        Aq = (torch.randn(9, L, D, device=dev) * 0.05).contiguous()
        Ar = torch.zeros(L, D, device=dev)
        ops2 = shards.kernel_ops(index, W, site_mask, k, Ar=Ar)
        idx2, _, (uniq, ucodes) = shards.sharded_neighbours(tok, k, ops2, aq_rows=Aq, want_codes=True)
        want2, _ = index.search(tok, W, site_mask, k, Aq=Aq, aq_period=9, Ar=Ar)
        assert torch.equal(idx2, want2)
        assert torch.equal(uniq, torch.unique(want2[want2 >= 0])) and torch.equal(ucodes, codes[uniq])
        done.append("sharded_neighbours (counts, codes + query offsets)")
        print(done[-1], flush=True)
        # one bucketed gradient all-reduce step over RCCL
        net = torch.nn.Sequential(torch.nn.Linear(32, 64), torch.nn.Tanh(), torch.nn.Linear(64, 16)).to(dev)
        fp = FlatParams(net.parameters(), mirror=False)
        bk = GradBucketer(fp, bucket_bytes=4096, always=True)
        assert bk.active and len(bk.buckets) >= 2
        net(torch.randn(8, 32, device=dev)).pow(2).sum().backward()
        before = fp.grad.clone()
        assert len(bk.handles) >= 1                        # launched from the accumulate hooks
        assert bk.finish() == 1.0
        torch.cuda.synchronize()
        assert torch.equal(fp.grad, before) and before.abs().sum() > 0
        done.append("GradBucketer async all_reduce")
        q.put(("ok", done))
    except Exception:
        q.put(("error", traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(140)
def test_rccl_world1_collectives():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    try:
        status, info = q.get(timeout=100)
    except Exception:                                  # queue.Empty: the child hung (e.g. in init)
        status, info = "hung", "no result from the nccl child within 100 s"
    finally:
        p.join(20)
        if p.is_alive():
            p.kill()
            p.join(10)
    assert status == "ok", info
    assert p.exitcode == 0
    print("\n".join(info))
