"""Where the wide-row block tail's cycles go (csrc/tailw.hip diagnostic instantiations; timing only,
their outputs are wrong): launch times at the bench shape (M = 512 x 1030) of
  base        tailw_kernel<0>
  W-cached    every W fragment load reads a 12 KiB cache-resident slice (bit 1: no L2-miss / HBM
              latency or L2 bandwidth in the weight stream)
  no-FFN1-LDS FFN1 steps read no B fragments (bit 2: FFN1 without its LDS traffic)
  both
and each one's per-wave phase stamps."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
sys.path.insert(0, os.path.dirname(__file__))
from src import kernels as K  # noqa: E402
from src import native as N  # noqa: E402
from tailw_micro_case import case  # noqa: E402

D = 384
M = int(os.environ.get("GM_M", 512 * 1030))
c = case(M, 1)
ts = K.tail_pack(c["w_o"], c["w1"], c["w2g"])
VARS = {"base": (1, 64), "early-resid": (17, 64), "no-split": (1, 0)}
if os.environ.get("DIAG_ALL"):
    VARS.update({"W-cached": (3, 64), "no-FFN1-LDS": (5, 64)})


def timeit(optv, reps=10):
    opt, split = optv
    xs = c["x"].clone()
    K.set_option("tail_split", split)
    K.set_option("tail_wide", opt)
    fn = lambda: K.tail_forward(c["att"], xs, ts, c["b_o"], c["g1"], c["be1"], c["vec"])
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    K.set_option("tail_wide", 1)
    return a.elapsed_time(b) / reps


for _ in range(20):
    timeit((1, 64), 1)
# correctness of the A/B arms (same arithmetic: bitwise equal outputs)
outs = {}
for name, (opt, split) in VARS.items():
    xs = c["x"].clone()
    K.set_option("tail_split", split)
    K.set_option("tail_wide", opt)
    K.tail_forward(c["att"], xs, ts, c["b_o"], c["g1"], c["be1"], c["vec"])
    outs[name] = xs
K.set_option("tail_wide", 1)
K.set_option("tail_split", 64)
print("bitwise equal to base: " + ", ".join(f"{n} {bool(torch.equal(o, outs['base']))}" for n, o in outs.items()),
      flush=True)
res = {k: [] for k in VARS}
for it in range(4):
    for name, opt in VARS.items():
        res[name].append(timeit(opt))
fl = 18.0 * M * D * D
for name, v in res.items():
    print(f"{name:12s} " + " ".join(f"{x:.4f}" for x in v) + f" ms  best {min(v):.4f} "
          f"({fl / min(v) / 1e9 / 2500:.3f} of 2.5 PF)", flush=True)

nwg = (M + 31) // 32                        # (32-row tiles of the split last round: more workgroups)
names = ["prologue", "out-projection", "LN1", "FFN (2304 MFMA)", "LN_f+LN2+stores"]
for name, (opt, split) in VARS.items():
    st = torch.zeros(nwg * 4 * 8, dtype=torch.int64, device="cuda")
    N.lib().snvrag_tail_stamps(st.data_ptr())
    xs = c["x"].clone()
    K.set_option("tail_split", split)
    K.set_option("tail_wide", opt + 1)
    K.tail_forward(c["att"], xs, ts, c["b_o"], c["g1"], c["be1"], c["vec"])
    torch.cuda.synchronize()
    K.set_option("tail_wide", 1)
    N.lib().snvrag_tail_stamps(None)
    s = st.view(nwg * 4, 8).cpu().numpy().astype(np.float64)
    s = s[s[:, 5] > 0]
    s = s[: ((M // 128) * 4)]                   # the 128-row tiles
    tot = s[:, 5] - s[:, 0]
    parts = [np.median(s[:, i + 1] - s[:, i]) for i in range(5)]
    print(f"{name:12s} stamps: " + ", ".join(f"{n} {p:.0f}" for n, p in zip(names, parts)) +
          f", total {np.median(tot):.0f} cyc; in FFN barriers {np.median(s[:, 6]):.0f}", flush=True)
