"""configs[1]'s train-mode retrieval and f32 loss across processes (r6 probe).  Unseeded, the
epoch-0 window masks (numpy's global RNG, the reference's semantics) differed per process and so
did the neighbours; tests/test_gpu_train.py _configs1_case now seeds them.  Prints the neighbour
hashes and the f32 loss of two constructions in this process (compare with another process)."""
import hashlib
import sys

sys.path[:0] = ["tests", "rag-snvbert_amd", "."]
import torch  # noqa: E402

import test_gpu_train as T  # noqa: E402
from src import autograd_ops as AO  # noqa: E402

h = lambda t: hashlib.md5(t.detach().cpu().numpy().tobytes()).hexdigest()[:12]
for rep in range(2):
    m, x = T._configs1_case()
    AO.set_train_precision(torch.float32)
    with torch.no_grad():
        L = float(T._configs1_loss(m, x))
    AO.set_train_precision(torch.bfloat16)
    print(rep, "rag_idx", h(x["rag_idx_h1"]), h(x["rag_idx_h2"]), "loss f32", L, flush=True)
