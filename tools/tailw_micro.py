"""Wide-row block tail (csrc/tailw.hip, option tail_wide) against tail_kernel (csrc/tail.hip):
correctness vs float64 torch on small ragged M, agreement with tail_kernel at the bench shape,
launch times (alternating, M = 512 x 1030), and the per-wave phase breakdown from the stamped
instantiation (tail_wide = 2)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402
from src import native as N  # noqa: E402

D = 384
dev, bf = "cuda", torch.bfloat16
F = torch.nn.functional
sys.path.insert(0, os.path.dirname(__file__))
from tailw_micro_case import case, ref  # noqa: E402


for M in (777, 128, 1, 4 * 1030 + 5):
    c = case(M, M)
    ts = K.tail_pack(c["w_o"], c["w1"], c["w2g"])
    r = ref(c)
    ew = (run(c, ts, 1).double() - r).abs()
    et = (run(c, ts, 0).double() - r).abs()
    print(f"M={M}: wide max|err| {ew.max().item():.4f} mean {ew.mean().item():.5f} | tail_kernel max "
          f"{et.max().item():.4f} mean {et.mean().item():.5f}", flush=True)

M = int(os.environ.get("GM_M", 512 * 1030))
c = case(M, 1)
ts = K.tail_pack(c["w_o"], c["w1"], c["w2g"])
ya, yb = run(c, ts, 1), run(c, ts, 0)
d = (ya.float() - yb.float()).abs()
print(f"bench shape M={M}: wide vs tail_kernel max|diff| {d.max().item():.4f} mean {d.mean().item():.6f} "
      f"differing {int((d > 0).sum())} of {d.numel()}", flush=True)
xs = c["x"].clone()


def timeit(wide, reps=10):
    K.set_option("tail_wide", wide)
    fn = lambda: K.tail_forward(c["att"], xs, ts, c["b_o"], c["g1"], c["be1"], c["vec"])
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    K.set_option("tail_wide", 0)
    return a.elapsed_time(b) / reps


fl = 18.0 * M * D * D
flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)


def timeit_cold(wide, reps=8):
    """each launch after a 512 MB write (weights and activations out of L2 / MALL, as in the
    encoder where QKV and attention stream GBs between two block tails); events around the tail only"""
    K.set_option("tail_wide", wide)
    tot = 0.0
    for _ in range(reps):
        flush.fill_(1)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        K.tail_forward(c["att"], xs, ts, c["b_o"], c["g1"], c["be1"], c["vec"])
        b.record()
        torch.cuda.synchronize()
        tot += a.elapsed_time(b)
    K.set_option("tail_wide", 0)
    return tot / reps


for _ in range(30):
    timeit(0, 1)
for it in range(2):
    for wide in (0, 1):
        print(f"cold caches: {'tailw (wide)' if wide else 'tail_kernel '} {timeit_cold(wide):.4f} ms", flush=True)
res = {0: [], 1: []}
for it in range(4):
    for wide in (0, 1):
        res[wide].append(timeit(wide))
for wide in (0, 1):
    v = res[wide]
    print(f"{'tailw (wide)' if wide else 'tail_kernel '}: " + " ".join(f"{x:.4f}" for x in v) +
          f" ms  best {min(v):.4f} = {fl / min(v) / 1e9:.0f} TFLOP/s ({fl / min(v) / 1e9 / 2500:.3f} of 2.5 PF)",
          flush=True)

# phase stamps (tail_wide = 2)
nwg = (M + 127) // 128
st = torch.zeros(nwg * 4 * 8, dtype=torch.int64, device=dev)
N.lib().snvrag_tail_stamps(st.data_ptr())
for _ in range(10):
    timeit(1, 1)
K.set_option("tail_wide", 2)
K.tail_forward(c["att"], xs, ts, c["b_o"], c["g1"], c["be1"], c["vec"])
torch.cuda.synchronize()
K.set_option("tail_wide", 0)
N.lib().snvrag_tail_stamps(None)
s = st.view(nwg * 4, 8).cpu().numpy().astype(np.float64)
names = ["prologue (att DMA, residual, tables)", "out-projection (288 MFMA)", "LN1 (2 barriers)",
         "FFN 6 rounds (2304 MFMA)", "LN_f + LN2 + stores"]
tot = s[:, 5] - s[:, 0]
for i, nm in enumerate(names):
    dd = s[:, i + 1] - s[:, i]
    print(f"  {nm:40s} median {np.median(dd):9.0f} cyc  p10 {np.percentile(dd, 10):9.0f}  p90 "
          f"{np.percentile(dd, 90):9.0f}  ({np.median(dd) / np.median(tot):.3f})", flush=True)
print(f"  {'wave total':40s} median {np.median(tot):9.0f} cyc  (MFMA floor 2592 x 32 = 82944)", flush=True)
