"""QKV projection on the 32x32 stream kernel (csrc/tail.hip PROJ mode) vs the stream GEMM (csrc/sgemm.hip, 4 and 8 waves) at the bench shape
(M = 512 x 1030, D = 384, N = 3D), plus the D -> 4D GELU projection on the stream GEMM: max |diff|
vs an fp64 reference on a small M, then launch times (HIP events)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

D, dev, bf = 384, "cuda", torch.bfloat16
g = torch.Generator(device="cpu").manual_seed(0)
w = (torch.randn(3 * D, D, generator=g) / D ** 0.5).to(dev, bf)
b = (0.1 * torch.randn(3 * D, generator=g)).to(dev)
ws = K.proj_pack(w)
for M in (777, 128 * 5 + 3):
    x = torch.randn(M, D, generator=g).to(dev, bf)
    o = K.proj_forward(x, ws, b, 3)
    ref = x.double() @ w.double().T + b.double()
    print(f"M={M} max|err| {(o.double() - ref).abs().max().item():.4f}", flush=True)
M = 512 * 1030
x = torch.randn(M, D, device=dev).to(bf)
out = torch.empty(M, 3 * D, device=dev, dtype=bf)


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return a.elapsed_time(e) / reps


fl = 2.0 * M * D * 3 * D
o1 = K.proj_forward(x, ws, b, 3, out=out).clone()
sgw, sgv = K.sgemm_pack(w), K.sgemm_vec(b)
o3 = K.sgemm(x, sgw, 3 * D, sgv)
print(f"proj vs sgemm max|diff| {(o1.float() - o3.float()).abs().max().item():.4f}", flush=True)
w4 = (torch.randn(4 * D, D, generator=g) / D ** 0.5).to(dev, bf)
b4 = (0.1 * torch.randn(4 * D, generator=g)).to(dev)
sg4, sv4 = K.sgemm_pack(w4), K.sgemm_vec(b4)
out4 = torch.empty(M, 4 * D, device=dev, dtype=bf)


def env(k, v):
    """SNVRAG_<NAME> -> the library option <name> (None: its default)."""
    name = k[len("SNVRAG_"):].lower()
    K.set_option(name, -1 if v is None and name.endswith("desync") else int(v or 0))


def proj_opt(wide):
    def fn():
        K.set_option("proj_wide", wide)
        K.proj_forward(x, ws, b, 3, out=out)
    return fn


K.set_option("proj_wide", 0)
o0 = K.proj_forward(x, ws, b, 3, out=out).clone()
K.set_option("proj_wide", 1)
o1w = K.proj_forward(x, ws, b, 3, out=out).clone()
print(f"wide proj vs tail.hip proj: max|diff| {(o1w.float() - o0.float()).abs().max().item():.4f}, "
      f"bitwise equal {torch.equal(o1w, o0)}", flush=True)
for it in range(3):
    for name, fn in (("proj wide (tailw.hip)", proj_opt(1)), ("sgemm", lambda: K.sgemm(x, sgw, 3 * D, sgv, out=out))):
        ms = timeit(fn)
        print(f"{name:24s} {ms:.4f} ms  {fl / ms / 1e9:.0f} TFLOP/s", flush=True)
K.set_option("proj_wide", 0)
for name, fn, e, f in (("proj (tail.hip)", lambda: K.proj_forward(x, ws, b, 3, out=out), None, fl),
                       ("sgemm", lambda: K.sgemm(x, sgw, 3 * D, sgv, out=out), None, fl),
                       ("gelu 4D", lambda: K.sgemm(x, sg4, 4 * D, sv4, act=1, out=out4), None, fl * 4 / 3)):
    env("SNVRAG_SG_WAVES4", e) if e else None
    ms = timeit(fn)
    print(f"{name:18s} {ms:.4f} ms  {f / ms / 1e9:.1f} TFLOP/s", flush=True)
for dz in ("0", "5000", "10000", "15000"):
    env("SNVRAG_SG_DESYNC", dz)
    ms = timeit(lambda: K.sgemm(x, sgw, 3 * D, sgv, out=out))
    print(f"sgemm desync {dz:6s} {ms:.4f} ms  {fl / ms / 1e9:.1f} TFLOP/s", flush=True)
    ms = timeit(lambda: K.sgemm(x, sg4, 4 * D, sv4, act=1, out=out4))
    print(f"gelu 4D desync {dz:6s} {ms:.4f} ms  {fl * 4 / 3 / ms / 1e9:.1f} TFLOP/s", flush=True)
env("SNVRAG_SG_DESYNC", None)
# the wave-count switch: env("SNVRAG_SG_WAVES4", "1") for 4 waves
print("(4-wave variant)" if os.environ.get("SNVRAG_SG_WAVES4") else "(8-wave variant)", flush=True)
