"""What HIP graphs would buy the bench step: capture (torch.cuda.CUDAGraph over the native
launches on the current stream) of (a) the eval forward with a fixed rag block and (b) the whole
step (kNN + rag_mean + forward), replay time against eager, and bitwise equality of the outputs.
Sizes are bench.py's defaults (configs[2]); run on the GPU box."""
import os
import sys
import time

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "rag-snvbert_amd"))
sys.argv = sys.argv[:1]
import bench  # noqa: E402
from src.dataset import synthetic  # noqa: E402
from src.dataset.vocab import WordVocab  # noqa: E402
from src.engine import engine_for  # noqa: E402
from src.model import build_model  # noqa: E402

args = bench.parse()
dev = torch.device("cuda:0")
torch.cuda.set_device(0)
vocab = WordVocab(synthetic.POPS)
torch.manual_seed(0)
model = build_model(len(vocab), args.dims, args.layers, args.heads).to(dev).eval()
eng = engine_for(model)
eng.set_dtype(torch.bfloat16)
wl = bench.build_workload(args, dev, vocab)
step = bench.make_step(wl, eng, args.k)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def probe(name, fn, key):
    for _ in range(3):
        ref = fn()
    torch.cuda.synchronize()
    ref = ref[key].clone()
    t_eager = timed(fn)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        fn()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    t0 = time.perf_counter()
    try:
        with torch.cuda.graph(g):
            out = fn()
    except Exception as e:  # noqa: BLE001 - report what blocks capture
        print(f"{name}: capture failed: {type(e).__name__}: {str(e)[:300]}", flush=True)
        torch.cuda.synchronize()
        return
    print(f"{name}: captured in {time.perf_counter() - t0:.2f} s", flush=True)
    t_graph = timed(g.replay)
    same = torch.equal(out[key], ref)
    diff = (out[key].float() - ref.float()).abs().max().item()
    print(f"{name}: eager {t_eager:.3f} ms, graph replay {t_graph:.3f} ms ({t_eager - t_graph:+.3f}); "
          f"outputs bitwise equal {same} (max |diff| {diff:.3g})", flush=True)


step()
torch.cuda.synchronize()
probe("forward", lambda: eng.forward(wl.x), "probs_h1")
probe("step (kNN + rag_mean + forward)", step, "probs_h1")
