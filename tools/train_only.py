"""The bench's training leg alone (bench.py train_bench: B = 24, window 512 -> L = 1030 tokens,
k = 8, d384/L12/H12) for profiling: warm-up steps, then TR_STEPS timed steps, reporting wall
ms/step next to the host time spent inside train_step (launch-bound if they agree and the
GPU kernel sum from rocprofv3 --stats is well below the wall)."""
import os
import sys
import time
from types import SimpleNamespace

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "rag-snvbert_amd")]
from src.dataset.embedding_rag_dataset import embedding_rag_collate_fn  # noqa: E402
from src.dataset.synthetic import make_rag_dataset  # noqa: E402
from src.main.pretrain_with_val_optimized import BERTTrainerWithValidationOptimized  # noqa: E402
from src.model import build_model  # noqa: E402

from src import autograd_ops  # noqa: E402

autograd_ops.set_blas_dx(os.environ.get("BLAS_DX", "0") == "1")    # A/B: hipBLASLt large-K GEMMs
dev = torch.device("cuda")
Bt, S = int(os.environ.get("TR_B", 24)), int(os.environ.get("TR_WINDOW", 512))
ds, vocab = make_rag_dataset(n_samples=Bt, n_sites=S, n_windows=1, n_ref_samples=5000, seed=7, name="train")
batch = embedding_rag_collate_fn([ds[i] for i in range(Bt)])
torch.manual_seed(0)
model = build_model(len(vocab), 384, 12, 12).to(dev)
tr = BERTTrainerWithValidationOptimized(model, None, None, vocab, lr=7.5e-5, warmup_steps=100, grad_accum_steps=1,
                                        log_freq=0)
tr.rag_train_dataset = ds
tr.rag_k = 8
for _ in range(int(os.environ.get("TR_WARM", 2))):
    tr.train_step(dict(batch))
torch.cuda.synchronize()
n = int(os.environ.get("TR_STEPS", 5))
host = 0.0
t0 = time.perf_counter()
for _ in range(n):
    h0 = time.perf_counter()
    loss = tr.train_step(dict(batch))
    host += time.perf_counter() - h0
torch.cuda.synchronize()
el = time.perf_counter() - t0
print(f"train B={Bt} window={S}: {el / n * 1e3:.2f} ms/step wall, {host / n * 1e3:.2f} ms/step host inside "
      f"train_step, loss {float(loss):.3f}", flush=True)

# phase split: the same step with a device sync after each phase (wall per phase) and the host
# time each phase takes to ENQUEUE (no sync) — a phase whose enqueue time approaches its wall
# time is launch/host bound
if os.environ.get("TR_SPLIT", "1") == "1":
    def phases(sync):
        t = {}
        data = dict(batch)
        tr.model.train()

        def mark(name, t0):
            if sync:
                torch.cuda.synchronize()
            t[name] = t.get(name, 0.0) + time.perf_counter() - t0

        t0 = time.perf_counter()
        data = ds.process_batch_retrieval(data, tr.embedding_layer, tr.device, k_retrieve=tr.rag_k)
        data = tr.to_device(data)
        mark("retrieval", t0)
        t0 = time.perf_counter()
        output = tr.model(data)
        total, parts = tr.loss(output, data)
        mark("forward+loss", t0)
        t0 = time.perf_counter()
        total.backward()
        mark("backward", t0)
        t0 = time.perf_counter()
        scale = tr.ddp.finish()
        tr.optim.step(grad_scale=scale)
        tr.optim_schedule.step()
        tr.optim.zero_grad()
        mark("optimizer", t0)
        return t
    torch.cuda.synchronize()
    for sync in (True, False):
        acc = {}
        for _ in range(3):
            torch.cuda.synchronize()
            for k, v in phases(sync).items():
                acc[k] = acc.get(k, 0.0) + v / 3
        torch.cuda.synchronize()
        print(("wall (synced) " if sync else "host enqueue  ") +
              "  ".join(f"{k} {v * 1e3:.2f} ms" for k, v in acc.items()), flush=True)
