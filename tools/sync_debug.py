"""Where the training step synchronises the host with the device: one bench-shape step under
torch.cuda.set_sync_debug_mode("warn"), each synchronising call reported once with its Python stack."""
import os
import sys
import traceback
import warnings

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "rag-snvbert_amd")]
from src.dataset.embedding_rag_dataset import embedding_rag_collate_fn  # noqa: E402
from src.dataset.synthetic import make_rag_dataset  # noqa: E402
from src.main.pretrain_with_val_optimized import BERTTrainerWithValidationOptimized  # noqa: E402
from src.model import build_model  # noqa: E402

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
for _ in range(2):
    tr.train_step(dict(batch))
torch.cuda.synchronize()
seen = {}


def show(message, category, filename, lineno, file=None, line=None):
    st = "".join(traceback.format_stack(limit=14)[:-2])
    key = (str(message)[:80], st[-600:])
    if key not in seen:
        seen[key] = 1
        print(f"--- {message}\n{st}", flush=True)


warnings.showwarning = show
torch.cuda.set_sync_debug_mode("warn")
tr.train_step(dict(batch))
torch.cuda.set_sync_debug_mode(0)
torch.cuda.synchronize()
print(f"{len(seen)} distinct synchronising call sites in one step", flush=True)
