"""What overlapping retrieval with the encoder would buy: the next batch's kNN search runs on a
second stream while the current batch's forward runs on the main stream (a serving pipeline),
against the sequential step of bench.py.  Checks the pipelined outputs bitwise against the
sequential ones.  Sizes are bench.py's defaults (configs[2]); run on the GPU box."""
import os
import sys

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "rag-snvbert_amd"))
sys.argv = sys.argv[:1]
import bench  # noqa: E402
from src import kernels as K  # noqa: E402
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
P = eng.packed()
B, L, D, k = wl.B, wl.L, P.D, args.k
Ar = eng.af_embedding(torch.from_numpy(wl.ref_af).to(dev)[None]).float()[0].contiguous()
search = bench.make_search(wl, eng, k)
step = bench.make_step(wl, eng, k)
blocks = [torch.empty(4 * B, L, D, device=dev, dtype=eng.dtype) for _ in range(2)]
side = torch.cuda.Stream()
main = torch.cuda.current_stream()


fwd_done = [None, None]                      # event after the forward that last read block j


def fill(i):
    """search + rag_mean of batch i into blocks[i % 2] on the side stream; returns its event"""
    if fwd_done[i % 2] is not None:
        side.wait_event(fwd_done[i % 2])     # the block's previous reader (forward i - 2) is done
    with torch.cuda.stream(side):
        idx, counts = search()
        K.rag_mean(idx, wl.index.codes, wl.S, P.W, P.pe, Ar, L, eng.dtype, out=blocks[i % 2][2 * B:],
                   counts=counts)
        ev = torch.cuda.Event()
        ev.record(side)
    return ev


def pipelined(n):
    outs = []
    side.wait_stream(main)
    ev = fill(0)
    for i in range(n):
        main.wait_event(ev)
        if i + 1 < n:
            ev = fill(i + 1)                 # runs beside forward i (waits only for forward i - 1)
        wl.x["rag_block"] = blocks[i % 2]
        o = eng.forward(wl.x)
        fwd_done[i % 2] = torch.cuda.Event()
        fwd_done[i % 2].record(main)
        outs.append(o["probs_h1"])
    main.wait_stream(side)
    return outs


def timed(fn, n=10):
    fn(2)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    fn(n)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n


seq = lambda n: [step()["probs_h1"] for _ in range(n)]
ref = seq(1)[0].clone()
torch.cuda.synchronize()
outs = pipelined(3)
torch.cuda.synchronize()
print("pipelined outputs bitwise equal to sequential:", all(torch.equal(o, ref) for o in outs), flush=True)
for _ in range(2):
    print(f"sequential {timed(seq):.3f} ms/step, pipelined {timed(pipelined):.3f} ms/step", flush=True)
