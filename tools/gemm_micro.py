"""GEMM micro-benchmark on the encoder's shapes (M = 128 sequences x 1030 tokens, d384).

Times each snvrag_linear_ex variant (row-panel deep/shallow, 128x128 tile) and, for a
practical ceiling, torch.matmul (hipBLASLt) on the same operands.  Prints one line per
case: ms, TFLOP/s, GB/s of compulsory traffic.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402
from src import native as N  # noqa: E402


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    M = int(os.environ.get("GM_M", 128 * 1030))
    D = 384
    dev = "cuda"
    dt = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, D, device=dev, generator=g).to(dt)
    h = torch.randn(M, 4 * D, device=dev, generator=g).to(dt)
    w = {(n, k): (torch.randn(n, k, device=dev, generator=g) / k ** 0.5).to(dt)
         for n, k in ((3 * D, D), (D, D), (4 * D, D), (D, 4 * D))}
    bias = {n: torch.randn(n, device=dev, generator=g) * 0.1 for n in (D, 3 * D, 4 * D)}
    lg, lb = torch.ones(D, device=dev), torch.zeros(D, device=dev)
    stats = torch.zeros(K.stat_tiles(4 * D), M, 2, device=dev)
    c1 = torch.randn(D, device=dev, generator=g)
    K.linear(x, w[(4 * D, D)], bias[4 * D], act=N.ACT_LRELU, slope=0.1, stats_out=stats)

    cases = {
        "qkv N1152 K384": (lambda: K.linear(x, w[(3 * D, D)], bias[3 * D]), M, 3 * D, D, 0),
        "oproj N384 K384 +resid+LN": (lambda: K.linear(x, w[(D, D)], bias[D], resid=x, ln=(lg, lb)), M, D, D, 1),
        "oproj N384 K384 plain": (lambda: K.linear(x, w[(D, D)], bias[D]), M, D, D, 0),
        "ffn1 N1536 K384 +lrelu+stats": (lambda: K.linear(x, w[(4 * D, D)], bias[4 * D], act=N.ACT_LRELU, slope=0.1,
                                                          stats_out=stats), M, 4 * D, D, 0),
        "ffn1 N1536 K384 +lrelu": (lambda: K.linear(x, w[(4 * D, D)], bias[4 * D], act=N.ACT_LRELU, slope=0.1),
                                   M, 4 * D, D, 0),
        "ffn1 N1536 K384 +stats": (lambda: K.linear(x, w[(4 * D, D)], bias[4 * D], stats_out=stats), M, 4 * D, D, 0),
        "oproj N384 K384 +resid": (lambda: K.linear(x, w[(D, D)], bias[D], resid=x), M, D, D, 1),
        "oproj N384 K384 +LN": (lambda: K.linear(x, w[(D, D)], bias[D], ln=(lg, lb)), M, D, D, 0),
        "ffn1 N1536 K384 plain": (lambda: K.linear(x, w[(4 * D, D)], bias[4 * D]), M, 4 * D, D, 0),
        "ffn1 N1536 K384 +gelu": (lambda: K.linear(x, w[(4 * D, D)], bias[4 * D], act=N.ACT_GELU), M, 4 * D, D, 0),
        "ffn2 N384 K1536 +rownorm+resid+LN": (lambda: K.linear(h, w[(D, 4 * D)], bias[D], act=N.ACT_LRELU, slope=0.1,
                                                               resid=x, ln=(lg, lb),
                                                               rownorm=(stats, K.stat_tiles(4 * D), 4 * D, c1)),
                                              M, D, 4 * D, 1),
        "ffn2 N384 K1536 plain": (lambda: K.linear(h, w[(D, 4 * D)], bias[D]), M, D, 4 * D, 0),
    }
    variants = [("rows", 0)] + ([("tile128", 1)] if os.environ.get("GM_ALL") else [])
    only = os.environ.get("GM_CASE")
    for name, (fn, m, n, k, extra) in cases.items():
        if only and not any(o in name for o in only.split(",")):
            continue
        flop = 2.0 * m * n * k
        byts = 2.0 * (m * k + n * k + m * n * (1 + extra)) if extra >= 0 else 2.0 * 2 * m * k
        for vn, env in variants:
            K.set_option("gemm_tile128", env)
            try:
                ms = timeit(fn)
            except Exception as e:  # the 128x128 tile has no fused-LN path
                print(f"{name:36s} {vn:8s} n/a ({str(e)[:60]})", flush=True)
                continue
            print(f"{name:36s} {vn:8s} {ms:8.3f} ms {flop / ms / 1e9:8.1f} TF/s {byts / ms / 1e6:8.1f} GB/s", flush=True)
        K.set_option("gemm_tile128", 0)
        if not os.environ.get("GM_TORCH"):
            continue
        if (n, k) not in w:
            continue
        a = h if k == 4 * D else x
        ww = w[(n, k)]
        ms = timeit(lambda: torch.matmul(a, ww.t()))
        print(f"{name:36s} {'torch':8s} {ms:8.3f} ms {flop / ms / 1e9:8.1f} TF/s {byts / ms / 1e6:8.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
