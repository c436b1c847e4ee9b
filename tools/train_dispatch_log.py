"""Where the training step's small ATen ops come from: one bench-shape train_step (B = 24, window
512, d384/L12) under a TorchDispatchMode that records every copy / add / cast / fill / cat / clone
with its shapes, dtypes and the innermost frames of this repository on the Python stack (ops the
autograd engine issues itself — gradient accumulation — show no repository frame)."""
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "rag-snvbert_amd")]
from src.dataset.embedding_rag_dataset import embedding_rag_collate_fn  # noqa: E402
from src.dataset.synthetic import make_rag_dataset  # noqa: E402
from src.main.pretrain_with_val_optimized import BERTTrainerWithValidationOptimized  # noqa: E402
from src.model import build_model  # noqa: E402

WANT = ("copy_", "add_", "add.", "_to_copy", "fill_", "zero_", "zeros", "cat", "clone", "mul.", "sum.", "index_put",
        "slice_backward", "gelu", "new_zeros", "empty", "where", "sub.", "div.")


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rows = collections.Counter()
        self.bytes = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = str(func)
        if any(w in name for w in WANT):
            ts = [a for a in args if isinstance(a, torch.Tensor)]
            shp = tuple((tuple(t.shape), str(t.dtype).replace("torch.", "")) for t in ts[:2])
            fr = [f"{os.path.basename(f.filename)}:{f.lineno}" for f in traceback.extract_stack()
                  if "rag-snvbert_amd" in f.filename or "/tools/" in f.filename][-3:]
            key = (name, shp, " <- ".join(reversed(fr)) or "(autograd engine)")
            self.rows[key] += 1
            self.bytes[key] += sum(t.numel() * t.element_size() for t in ts)
        return out


dev = torch.device("cuda")
ds, vocab = make_rag_dataset(n_samples=24, n_sites=512, n_windows=1, n_ref_samples=5000, seed=7, name="train")
batch = embedding_rag_collate_fn([ds[i] for i in range(24)])
torch.manual_seed(0)
model = build_model(len(vocab), 384, 12, 12).to(dev)
tr = BERTTrainerWithValidationOptimized(model, None, None, vocab, lr=7.5e-5, warmup_steps=100, grad_accum_steps=1,
                                        log_freq=0)
tr.rag_train_dataset = ds
tr.rag_k = 8
for _ in range(2):
    tr.train_step(dict(batch))
torch.cuda.synchronize()
log = Log()
with log:
    tr.train_step(dict(batch))
torch.cuda.synchronize()
print("by calls: calls  bytes (MB)  op  shapes  origin")
for key, n in sorted(log.rows.items(), key=lambda kv: -kv[1])[:40]:
    name, shp, fr = key
    print(f"{n:5d} {log.bytes[key] / 1e6:9.1f}  {name[:28]:28s} {str(shp)[:90]:90s} {fr}", flush=True)
print("bytes touched (MB)  calls  op  shapes  origin")
for key, b in sorted(log.bytes.items(), key=lambda kv: -kv[1])[:60]:
    name, shp, fr = key
    print(f"{b / 1e6:9.1f} {log.rows[key]:5d}  {name[:28]:28s} {str(shp)[:90]:90s} {fr}", flush=True)
