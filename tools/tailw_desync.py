"""Wide-row block tail (csrc/tailw.hip): launch time at the bench shape (M = 512 x 1030) for
first-round stagger steps (option tail_desync, cycles per phase step; -1 = the library default),
alternated so box drift spreads over all settings."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

D, dev, bf = 384, "cuda", torch.bfloat16
M = int(os.environ.get("GM_M", 512 * 1030))
g = torch.Generator(device="cpu").manual_seed(1)
r = lambda *s, sc=1.0: (sc * torch.randn(*s, generator=g)).to(dev)
x, att = r(M, D).to(bf), r(M, D, sc=0.5).to(bf)
w_o, w1 = (r(D, D) / D ** 0.5).to(bf), (r(4 * D, D) / D ** 0.5).to(bf)
w2 = r(D, 4 * D) / (4 * D) ** 0.5
b_o, b1, b2 = r(D, sc=0.1), r(4 * D, sc=0.1), r(D, sc=0.1)
g1, be1, gf, bff = 1 + r(D, sc=0.2), r(D, sc=0.1), 1 + r(4 * D, sc=0.2), r(4 * D, sc=0.1)
g2, be2 = 1 + r(D, sc=0.2), r(D, sc=0.1)
w2g, b2g, _ = K.fold_layernorm(w2, b2, gf, bff, bf)
vec = K.ffn_vec(b1, b2g, w2g, g2, be2)
ts = K.tail_pack(w_o, w1, w2g)
K.set_option("tail_wide", 1)


def timeit(dz, reps=10):
    K.set_option("tail_desync", dz)
    fn = lambda: K.tail_forward(att, x, ts, b_o, g1, be1, vec)
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for _ in range(20):
    timeit(-1, 1)
vals = [int(v) for v in os.environ.get("DZ", "0,10000,20000,-1,30000,40000").split(",")]
res = {v: [] for v in vals}
for it in range(4):
    for v in vals:
        res[v].append(timeit(v))
for v in vals:
    print(f"tail_desync {v:6d}: " + " ".join(f"{t:.4f}" for t in res[v]) + f"  median {sorted(res[v])[len(res[v]) // 2]:.4f} ms",
          flush=True)
