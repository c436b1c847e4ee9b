"""HBM read / write / copy bandwidth with torch ops (sanity ceiling for the GEMM stores)."""
import torch


def timeit(fn, reps=20):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for mb in (100, 400, 1600):
    n = mb * (1 << 20) // 2
    x = torch.randn(n, device="cuda").to(torch.bfloat16)
    y = torch.empty_like(x)
    t = timeit(lambda: y.fill_(1.0)); print(f"{mb}MB fill  {mb / 1024 / t * 1e3 / 1e3 * 1.073741824:.2f} TB/s")
    t = timeit(lambda: y.copy_(x)); print(f"{mb}MB copy  {2 * mb / 1024 / t * 1.073741824:.2f} TB/s")
    t = timeit(lambda: x.sum()); print(f"{mb}MB sum   {mb / 1024 / t * 1.073741824:.2f} TB/s")
