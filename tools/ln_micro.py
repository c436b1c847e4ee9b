"""LayerNorm training kernels at the training shapes (M = 2 * 24 * 1030 rows): forward and
backward per launch for N = 384 (block norms, residual dropout + activation) and N = 1536 (the
FFN norm with its input activation), and the bytes they move."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

M = int(os.environ.get("M", 2 * 24 * 1030))


def tm(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for N, mode, rows1 in ((384, "resid", 1), (384, "resid", 0), (1536, "act_x", 0), (384, "plain", 1), (384, "plain", 0)):
    K.set_option("ln_rows1", rows1)           # 1: one row per wave (the pre-r4 kernels)
    x = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    r = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    g = torch.ones(N, device="cuda")
    b = torch.zeros(N, device="cuda")
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    if mode == "resid":
        kw = dict(p_r=0.1, p_out=0.19, seed=5, slope_r=0.1)
        y, s, st = K.ln_fwd_train(x, r, g, b, 1e-5, **kw)
        f = tm(lambda: K.ln_fwd_train(x, r, g, b, 1e-5, **kw))
        bw = tm(lambda: K.ln_bwd(dy, s, st, g, 0.1, 0.19, 5, slope_r=0.1, r_pre=r))
        nb = 6 * M * N * 2
    elif mode == "act_x":
        y, s, st = K.ln_fwd_train(x, None, g, b, 1e-5, slope_x=0.1)
        f = tm(lambda: K.ln_fwd_train(x, None, g, b, 1e-5, slope_x=0.1))
        bw = tm(lambda: K.ln_bwd(dy, s, st, g, slope_x=0.1))
        nb = 3 * M * N * 2
    else:
        y, s, st = K.ln_fwd_train(x, None, g, b, 1e-5, p_out=0.1, seed=3)
        f = tm(lambda: K.ln_fwd_train(x, None, g, b, 1e-5, p_out=0.1, seed=3))
        bw = tm(lambda: K.ln_bwd(dy, s, st, g, 0.0, 0.1, 3))
        nb = 3 * M * N * 2
    print(f"N={N} {mode} rows1={rows1}: fwd {f:.1f} us  bwd {bw:.1f} us ({nb / bw / 1e3:.0f} GB/s)", flush=True)
