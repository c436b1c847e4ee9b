"""torch.profiler over the bench's training step (B = 24, window 512, d384/L12): the ATen ops
(and the HIP-kernel autograd nodes) by device time, to find the elementwise work left outside the
hand-written kernels."""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "rag-snvbert_amd")]
from src.dataset.embedding_rag_dataset import embedding_rag_collate_fn  # noqa: E402
from src.dataset.synthetic import make_rag_dataset  # noqa: E402
from src.main.pretrain_with_val_optimized import BERTTrainerWithValidationOptimized  # noqa: E402
from src.model import build_model  # noqa: E402

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
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    for _ in range(3):
        tr.train_step(dict(batch))
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=45,
                                                           max_name_column_width=40, max_shapes_column_width=60))
# ATen ops only (the Python-level torch work left around the HIP kernels), by device time incl. children
rows = [e for e in prof.key_averages(group_by_input_shape=True) if e.key.startswith("aten::")]
rows.sort(key=lambda e: -e.device_time_total)
print("\nATen ops by device time (ms per step, calls per step, shapes)")
for e in rows[:60]:
    print(f"{e.device_time_total / 3e3:8.3f} ms {e.count / 3:6.1f}  {e.key:28s} {str(e.input_shapes)[:110]}")

if os.environ.get("STACKS"):
    # where the small glue ops come from: the Python stacks of the top ATen callers
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof2:
        tr.train_step(dict(batch))
        torch.cuda.synchronize()
    want = {"aten::cat", "aten::zeros", "aten::copy_", "aten::add_", "aten::_to_copy", "aten::clone", "aten::fill_"}
    rows = [e for e in prof2.key_averages(group_by_input_shape=True, group_by_stack_n=6) if e.key in want]
    rows.sort(key=lambda e: -e.device_time_total)
    print("\nGlue ops by Python stack (one step: device ms, calls)")
    for e in rows[:40]:
        st = " <- ".join(s.split("/")[-1] for s in e.stack[:6]) or "(no Python stack: autograd engine)"
        print(f"{e.device_time_total / 1e3:7.3f} ms {e.count:4d}  {e.key:16s} {str(e.input_shapes)[:60]} {st[:260]}")

if os.environ.get("PARENTS"):
    # glue ops attributed to the autograd node (or forward op) that issued them: the nearest CPU
    # ancestor that is an autograd evaluate_function / custom Function backward / top-level op
    import collections
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof3:
        tr.train_step(dict(batch))
        torch.cuda.synchronize()
    want = ("aten::cat", "aten::zeros", "aten::copy_", "aten::add_", "aten::add", "aten::_to_copy", "aten::clone",
            "aten::fill_", "aten::zero_", "aten::mul", "aten::sum", "aten::slice_backward", "aten::gelu",
            "aten::gelu_backward", "aten::index_put_", "aten::where", "aten::mean")
    agg = collections.defaultdict(lambda: [0.0, 0])
    for e in prof3.events():
        if e.name not in want:
            continue
        # only top-level glue (not a copy_ inside _to_copy etc.)
        if e.cpu_parent is not None and e.cpu_parent.name in want:
            continue
        p, anc = e.cpu_parent, "(top level)"
        while p is not None:
            if p.name.startswith("autograd::engine::evaluate_function") or "Backward" in p.name or \
                    p.name.startswith("_Hip") or p.name.startswith("_Nbr"):
                anc = p.name.replace("autograd::engine::evaluate_function: ", "")
                break
            p = p.cpu_parent
        shp = str(e.input_shapes)[:70] if e.input_shapes else ""
        key = (e.name, anc, shp)
        agg[key][0] += getattr(e, "device_time_total", 0.0)
        agg[key][1] += 1
    print("\nGlue ops by issuing autograd node (one step: device ms, calls)")
    for (n, a, s), (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:60]:
        print(f"{t / 1e3:7.3f} ms {c:4d}  {n:22s} {a[:40]:40s} {s}")
