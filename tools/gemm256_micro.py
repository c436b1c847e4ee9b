"""Large-K -> 384 GEMMs of training (w_2 forward, the K = 1152 / 1536 dX GEMMs) at M = 49 440:
the wide-row GEMM (csrc/gemm256.hip) vs hipBLASLt (torch.addmm) vs the row-panel GEMM."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

dev, bf = "cuda", torch.bfloat16
M = int(os.environ.get("GM_M", 49440))


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


x = torch.randn(4096, 4096, device=dev)
for _ in range(50):                                   # clock warm-up
    x @ x
for Kd in (1536, 1152):
    a = torch.randn(M, Kd, device=dev).to(bf)
    w = (torch.randn(384, Kd, device=dev) / Kd ** 0.5).to(bf)
    b = torch.randn(384, device=dev)
    r = torch.randn(M, 384, device=dev).to(bf)
    wp = K.gemm256_pack(w)
    out = torch.empty(M, 384, device=dev, dtype=bf)
    fl = 2.0 * M * 384 * Kd
    ref = torch.addmm(b.to(bf), a, w.t())
    y = K.gemm256(a, wp, 384, bias=b, out=out)
    print(f"K={Kd}: max|gemm256 - hipBLASLt| {(y.float() - ref.float()).abs().max().item():.4f}", flush=True)
    K.set_option("g2_variant", 4)
    y1 = K.gemm256(a, wp, 384, bias=b)
    K.set_option("g2_variant", 0)
    print(f"  v2 == v1 bitwise: {torch.equal(y1, y)}", flush=True)
    for name, fn in (("gemm256 +bias", lambda: K.gemm256(a, wp, 384, bias=b, out=out)),
                     ("gemm256 +resid", lambda: K.gemm256(a, wp, 384, resid=r, out=out)),
                     ("hipBLASLt addmm", lambda: torch.addmm(b.to(bf), a, w.t())),
                     ("hipBLASLt mm", lambda: torch.mm(a, w.t())),
                     ("row-panel linear", lambda: K.linear(a, w, b)),
                     ("gemm256 again", lambda: K.gemm256(a, wp, 384, bias=b, out=out)),
                     ("diag: no A loads", lambda: (K.set_option("g2_variant", 1),
                                                   K.gemm256(a, wp, 384, bias=b, out=out))),
                     ("diag: no MFMA", lambda: (K.set_option("g2_variant", 2),
                                                K.gemm256(a, wp, 384, bias=b, out=out))),
                     ("v1 (W via LDS)", lambda: (K.set_option("g2_variant", 4),
                                                 K.gemm256(a, wp, 384, bias=b, out=out))),
                     ("gemm256 (3rd)", lambda: (K.set_option("g2_variant", 0),
                                                K.gemm256(a, wp, 384, bias=b, out=out))),
                     ("groups 8 (256 rows)", lambda: (K.set_option("g2_groups", 8),
                                                      K.gemm256(a, wp, 384, bias=b, out=out))),
                     ("groups 6 (192 rows)", lambda: (K.set_option("g2_groups", 6),
                                                      K.gemm256(a, wp, 384, bias=b, out=out))),
                     ("groups 5 (160 rows)", lambda: (K.set_option("g2_groups", 5),
                                                      K.gemm256(a, wp, 384, bias=b, out=out))),
                     ("groups 4 (128 rows)", lambda: (K.set_option("g2_groups", 4),
                                                      K.gemm256(a, wp, 384, bias=b, out=out))),
                     ("default (4th)", lambda: (K.set_option("g2_groups", 0),
                                                K.gemm256(a, wp, 384, bias=b, out=out)))):
        ms = timeit(fn)
        print(f"  {name:20s} {ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TFLOP/s", flush=True)

# ---- stamps (g2_variant 3): per-wave cycles, in-kernel clock
import numpy as np  # noqa: E402
from src import native as NN  # noqa: E402

Kd = 1536
a = torch.randn(M, Kd, device=dev).to(bf)
w = (torch.randn(384, Kd, device=dev) / Kd ** 0.5).to(bf)
wp = K.gemm256_pack(w)
out = torch.empty(M, 384, device=dev, dtype=bf)
nwg = (M + 127) // 128
st = torch.zeros(nwg * 4 * 8, dtype=torch.int64, device=dev)
for _ in range(200):
    K.gemm256(a, wp, 384, out=out)
for var, nm in ((3, "v2"), (7, "v1")):
    st.zero_()
    NN.lib().snvrag_tail_stamps(st.data_ptr())
    K.set_option("g2_variant", var)
    K.gemm256(a, wp, 384, out=out)
    torch.cuda.synchronize()
    K.set_option("g2_variant", 0)
    NN.lib().snvrag_tail_stamps(None)
    s = st.view(nwg * 4, 8).cpu().numpy().astype(np.float64)
    clk = (s[:, 4] - s[:, 0]) / np.maximum(s[:, 5] - s[:, 1], 1) * 0.1
    tot = s[:, 4] - s[:, 0]
    print(f"{nm} stamped K={Kd}: clock median {np.median(clk):.3f} GHz; wave total median {np.median(tot):.0f} cyc "
          f"(MFMA floor {Kd // 64 * 96 * 32})", flush=True)
    for nm, d in (("prologue to first slab", s[:, 2] - s[:, 0]), ("K loop", s[:, 3] - s[:, 2]),
                  ("epilogue", s[:, 4] - s[:, 3]), ("  slab waits in loop", s[:, 6]), ("  B-fragment phase", s[:, 7])):
        print(f"  {nm:26s} median {np.median(d):9.0f}  p10 {np.percentile(d, 10):9.0f}  p90 {np.percentile(d, 90):9.0f}",
              flush=True)
    r0, r1 = s[:, 1].reshape(nwg, 4).min(1), s[:, 5].reshape(nwg, 4).max(1)
    print(f"  launch span {(r1.max() - r0.min()) / 100:.1f} us; workgroup lifetimes median {np.median(r1 - r0) / 100:.1f} us",
          flush=True)
