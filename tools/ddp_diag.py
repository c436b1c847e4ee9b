"""Per-sample record of the two-rank vs one-process entry-point run of
tests/test_gpu_ddp.py::test_train_main_two_ranks_global_metrics_and_early_stop.

Each run records, for every train/val batch, per sample (keyed by its token / mask bytes): the
retrieved neighbour indices of both haplotypes, the per-sample focal-loss parts and the output
probabilities at the masked sites.  The report names the first samples whose neighbours or loss
parts differ between the runs.

  python tools/ddp_diag.py OUTDIR
"""
import hashlib
import os
import socket
import tempfile
import sys

import numpy as np
import torch
import torch.multiprocessing as mp

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "rag-snvbert_amd")]

ARGS = ["--synthetic", "8", "--synthetic_sites", "300", "--synthetic_windows", "1", "--synthetic_ref", "40",
        "--dims", "128", "--layers", "2", "--attn_heads", "4", "--epochs", "3", "--patience", "1",
        "--lr", "0", "--dropout", "0", "--grad_accum_steps", "1", "--rag_k", "4", "--log_freq", "0",
        "--warmup_steps", "1"]


def _install(rec):
    from src.main import pretrain_with_val_optimized as T
    cls = T.BERTTrainerWithValidationOptimized
    orig_epoch = cls._run_epoch
    state = {"epoch": -1, "train": True}

    def run_epoch(self, epoch, dataloader, train=True):
        state["epoch"], state["train"] = epoch, train
        return orig_epoch(self, epoch, dataloader, train)

    orig_loss = cls.loss

    def loss(self, output, data):
        r = orig_loss(self, output, data)
        with torch.no_grad():
            m = data["mask"].bool()
            B = m.shape[0]
            for i in range(B):
                key = hashlib.sha1(data["hap_1"][i].cpu().numpy().tobytes() + data["hap_2"][i].cpu().numpy().tobytes()
                                   + data["mask"][i].cpu().numpy().tobytes()).hexdigest()[:16]
                mi = m[i:i + 1]
                l1 = self.hap_criterion(output[0][i:i + 1], data["hap_1_label"][i:i + 1], mi)
                l2 = self.hap_criterion(output[1][i:i + 1], data["hap_2_label"][i:i + 1], mi)
                lg = self.gt_criterion(output[2][i:i + 1], data["gt_label"][i:i + 1], mi)
                sel = mi[0]
                rec.append(dict(epoch=state["epoch"], train=state["train"], key=key,
                                idx1=data["rag_idx_h1"][i].cpu().numpy().copy() if "rag_idx_h1" in data else None,
                                idx2=data["rag_idx_h2"][i].cpu().numpy().copy() if "rag_idx_h2" in data else None,
                                parts=np.array([float(l1), float(l2), float(lg)], np.float64),
                                p1=output[0][i][sel].float().cpu().numpy(), p2=output[1][i][sel].float().cpu().numpy(),
                                pg=output[2][i][sel].float().cpu().numpy(), batch_parts=[float(p) for p in r[1]]))
        return r
    cls._run_epoch = run_epoch
    cls.loss = loss


def _save(rec, path):
    import pickle
    with open(path, "wb") as f:     # our own records only (tool output, never reference data)
        pickle.dump(rec, f)


def _worker(rank, world, port, out, tag):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK="0")
    import torch.distributed as dist
    rec = []
    _install(rec)
    from src import train_embedding_rag
    try:
        train_embedding_rag.main(ARGS + ["--train_batch_size", "2", "--val_batch_size", "1", "--dist_backend", "gloo",
                                         "--panel", "sharded", "--metrics_csv", os.path.join(out, f"{tag}.csv"),
                                         "--output_path", os.path.join(tempfile.mkdtemp(), "model")])
    finally:
        _save(rec, os.path.join(out, f"{tag}_rank{rank}.pkl"))
        if dist.is_initialized():
            dist.destroy_process_group()


def _load(path):
    import pickle
    with open(path, "rb") as f:
        return pickle.load(f)


def _run_ddp(out, tag):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    ps = [ctx.Process(target=_worker, args=(r, 2, port, out, tag)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(400)
    return _load(os.path.join(out, f"{tag}_rank0.pkl")) + _load(os.path.join(out, f"{tag}_rank1.pkl"))


def _run_single(out, tag):
    rec = []
    _install(rec)
    from src import train_embedding_rag
    train_embedding_rag.main(ARGS + ["--train_batch_size", "4", "--val_batch_size", "2",
                                     "--metrics_csv", os.path.join(out, f"{tag}.csv"),
                                     "--output_path", os.path.join(tempfile.mkdtemp(), "model")])
    _save(rec, os.path.join(out, f"{tag}.pkl"))
    return rec


def compare(a, b, name):
    by = {}
    for r in b:
        by[(r["epoch"], r["train"], r["key"])] = r
    n_bad = 0
    tot = {}
    for r in a:
        k = (r["epoch"], r["train"], r["key"])
        s = by.get(k)
        tot.setdefault(k[:2], [0.0, 0.0])
        tot[k[:2]][0] += r["parts"].sum()
        if s is None:
            print(name, "no record for", k)
            continue
        tot[k[:2]][1] += s["parts"].sum()
        same_idx = np.array_equal(r["idx1"], s["idx1"]) and np.array_equal(r["idx2"], s["idx2"])
        dp = np.abs(r["parts"] - s["parts"]).max()
        dprob = max(np.abs(r["p1"] - s["p1"]).max(), np.abs(r["p2"] - s["p2"]).max(), np.abs(r["pg"] - s["pg"]).max())
        if not same_idx or dp > 1e-6 * max(1.0, np.abs(s["parts"]).max()):
            n_bad += 1
            print(f"{name} MISMATCH epoch {k[0]} train {k[1]} key {k[2]}: idx equal {same_idx} parts {r['parts']} vs "
                  f"{s['parts']} max|dprob| {dprob:.3e}")
            if not same_idx:
                print("   a idx1", r["idx1"].tolist(), "idx2", r["idx2"].tolist())
                print("   b idx1", s["idx1"].tolist(), "idx2", s["idx2"].tolist())
    for k, v in sorted(tot.items()):
        print(name, "epoch/train", k, "sum of per-sample parts a %.6f b %.6f" % tuple(v))
    print(name, "mismatching samples:", n_bad, flush=True)


def main(out, n_ddp=3, n_single=2):
    os.makedirs(out, exist_ok=True)
    runs = {}
    for i in range(n_ddp):
        runs[f"ddp{i}"] = _run_ddp(out, f"ddp{i}")
        print(open(os.path.join(out, f"ddp{i}.csv")).read(), flush=True)
    for i in range(n_single):
        runs[f"one{i}"] = _run_single(out, f"one{i}")
        print(open(os.path.join(out, f"one{i}.csv")).read(), flush=True)
    for name, rec in runs.items():
        if name != "one0":
            compare(rec, runs["one0"], f"[{name} vs one0]")


if __name__ == "__main__":
    main(sys.argv[1], *map(int, sys.argv[2:]))
