"""32x32-MFMA block tail (csrc/tail.hip): correctness against a float64 torch reference on a small M,
then launch times of its variants at the bench shape (M = 512 x 1030), and the per-wave phase
breakdown from the stamped diagnostic instantiation (s_memtime / s_memrealtime)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402

D = 384
dev, bf = "cuda", torch.bfloat16
K.set_option("tail_wide", 0)                         # this tool measures tail_kernel / tailp_kernel
F = torch.nn.functional


def case(M, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    r = lambda *s, sc=1.0: (sc * torch.randn(*s, generator=g)).to(dev)
    x, att = r(M, D).to(bf), r(M, D, sc=0.5).to(bf)
    w_o, w1 = (r(D, D) / D ** 0.5).to(bf), (r(4 * D, D) / D ** 0.5).to(bf)
    w2 = r(D, 4 * D) / (4 * D) ** 0.5
    b_o, b1, b2 = r(D, sc=0.1), r(4 * D, sc=0.1), r(D, sc=0.1)
    g1, be1 = 1 + r(D, sc=0.2), r(D, sc=0.1)
    gf, bff = 1 + r(4 * D, sc=0.2), r(4 * D, sc=0.1)
    g2, be2 = 1 + r(D, sc=0.2), r(D, sc=0.1)
    w2g, b2g, _ = K.fold_layernorm(w2, b2, gf, bff, bf)
    vec = K.ffn_vec(b1, b2g, w2g, g2, be2)
    return dict(x=x, att=att, w_o=w_o, w1=w1, w2=w2, w2g=w2g, b_o=b_o, b1=b1, b2=b2, g1=g1, be1=be1, gf=gf,
                bff=bff, g2=g2, be2=be2, vec=vec)


def ref(c, pre=True):
    xd = c["x"].double()
    if pre:
        x1 = F.layer_norm(xd + c["att"].double() @ c["w_o"].double().T + c["b_o"].double(), (D,),
                          c["g1"].double(), c["be1"].double(), 1e-5)
    else:
        x1 = xd
    h = F.leaky_relu(x1 @ c["w1"].double().T + c["b1"].double(), 0.1)
    hn = F.layer_norm(h, (4 * D,), c["gf"].double(), c["bff"].double(), 1e-5)
    f = F.leaky_relu(hn @ c["w2"].double().T + c["b2"].double(), 0.1)
    return F.layer_norm(x1 + f, (D,), c["g2"].double(), c["be2"].double(), 1e-5)


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


c = case(777 + 128 * 3)
ts = K.tail_pack(c["w_o"], c["w1"], c["w2g"])
xx = c["x"].clone()
K.tail_forward(c["att"], xx, ts, c["b_o"], c["g1"], c["be1"], c["vec"])
e = (xx.double() - ref(c, True)).abs()
print(f"tail PRE   max|err| {e.max().item():.4f} mean {e.mean().item():.5f}", flush=True)
o = K.tail_ffn_forward(c["x"], ts, c["vec"])
e = (o.double() - ref(c, False)).abs()
print(f"tail FFN   max|err| {e.max().item():.4f} mean {e.mean().item():.5f}", flush=True)

M = int(os.environ.get("GM_M", 512 * 1030))
c = case(M, 1)
ts = K.tail_pack(c["w_o"], c["w1"], c["w2g"])
xs = c["x"].clone()
out = torch.empty_like(c["x"])
fl9, fl8 = 18.0 * M * D * D, 16.0 * M * D * D
def tail_var(v, desync=-1, persist=0):
    def fn():
        K.set_option("tail_variant", int(v))
        K.set_option("tail_persist", int(persist))
        if desync < 0:
            K.set_option("tail_desync", -1)         # the library default
        else:
            K.set_option("tail_desync", int(desync))
        K.tail_forward(c["att"], xs, ts, c["b_o"], c["g1"], c["be1"], c["vec"])
    return fn


for _ in range(30):                                  # clock warm-up before the first timing
    tail_var(0)()
# persistent kernel (default) == tail_kernel bit for bit at the bench shape
ya, yb = c["x"].clone(), c["x"].clone()
tail_var(0, persist=1)()
K.tail_forward(c["att"], ya, ts, c["b_o"], c["g1"], c["be1"], c["vec"])
tail_var(0)()
K.tail_forward(c["att"], yb, ts, c["b_o"], c["g1"], c["be1"], c["vec"])
print(f"persistent vs tail_kernel at M = {M}: bitwise equal {torch.equal(ya, yb)}, "
      f"differing outputs {int((ya != yb).sum())} of {ya.numel()}", flush=True)
for name, fn, fl in (
        ("tailp (persistent)", tail_var(0, persist=1), fl9),
        ("tailp no desync", tail_var(0, 0, 1), fl9),
        ("tail_kernel PRE (PF 8, default)", tail_var(0), fl9),
        ("tail_kernel PRE PF 4", tail_var(1), fl9),
        ("tailp (again)", tail_var(0, persist=1), fl9),
        ("tail.hip PRE residual at group 3", tail_var(5), fl9),
        ("tail_kernel PRE PF 8 (again)", tail_var(0), fl9),
        ("tail.hip PRE no-DMA (diag)", tail_var(2), fl9),
        ("tail.hip PRE no sched groups", tail_var(3), fl9),
        ("tail.hip PRE no desync", tail_var(0, 0, 0), fl9),
        ("tail.hip FFN only", lambda: (K.set_option("tail_variant", 0),
                                       K.tail_ffn_forward(c["x"], ts, c["vec"], out=out)), fl8)):
    ms = timeit(fn)
    print(f"{name:22s} {ms:.4f} ms  {fl / ms / 1e9:.1f} TFLOP/s", flush=True)

# ---- phase stamps (SNVRAG_TAIL_VARIANT=4: the PRE kernel with s_memtime stamps per wave)
import numpy as np  # noqa: E402
from src import native as N  # noqa: E402

nwg = (M + 127) // 128
st = torch.zeros(nwg * 4 * 10, dtype=torch.int64, device=dev)
N.lib().snvrag_tail_stamps(st.data_ptr())
for _ in range(20):                                  # warm the clock up on the default kernel
    tail_var(0)()
tail_var(4, int(os.environ.get("TM_DESYNC", "-1")))()
torch.cuda.synchronize()
N.lib().snvrag_tail_stamps(None)
K.set_option("tail_variant", 0)
s = st.view(nwg * 4, 10).cpu().numpy().astype(np.float64)
names = ["prologue (act loads + 8 slabs)", "out-projection (864 MFMA)", "LN1", "FFN (1728 MFMA)",
         "FFN end -> ring free (vmcnt 0 + barrier + vec tables)", "LN2 + stores (+ vmcnt 0)"]
clk = (s[:, 7] - s[:, 1]) / np.maximum(s[:, 8] - s[:, 0], 1) * 0.1     # GHz (realtime = 100 MHz)
print(f"stamped launch: {nwg} workgroups; in-kernel clock median {np.median(clk):.3f} GHz", flush=True)
tot = s[:, 7] - s[:, 1]
for i, nm in enumerate(names):
    d = s[:, i + 2] - s[:, i + 1]
    print(f"  {nm:55s} median {np.median(d):9.0f} cyc  p10 {np.percentile(d, 10):9.0f}  p90 {np.percentile(d, 90):9.0f}"
          f"  ({np.median(d) / np.median(tot):.3f} of the wave)", flush=True)
print(f"  {'wave total':55s} median {np.median(tot):9.0f} cyc  (MFMA floor 2592 x 32 = 82944)", flush=True)
r0 = s[:, 0].reshape(nwg, 4).min(1)
r1 = s[:, 8].reshape(nwg, 4).max(1)
span = (r1.max() - r0.min())
busy = (r1 - r0).sum() / (256 * span)
print(f"  workgroup residency: span {span / 100:.1f} us, sum of workgroup lifetimes / (256 CUs x span) = {busy:.3f}",
      flush=True)
order = np.sort(r0 - r0.min()) / 100
print("  workgroup start times (us) at ranks 0/256/512/.../end: " +
      " ".join(f"{order[i]:.1f}" for i in range(0, nwg, 256)) + f" | last {order[-1]:.1f}", flush=True)

# ---- persistent kernel phase stamps (SNVRAG_TAIL_VARIANT=7): the last tile of every wave
import ctypes  # noqa: E402
nbuf = ctypes.create_string_buffer(64)
n_cu = N.lib().snvrag_device_info(0, nbuf, 64)
G = min((M + 127) // 128, n_cu)
print(f"device {nbuf.value.decode()}: {n_cu} CUs -> persistent grid {G}", flush=True)
stp = torch.zeros(max(G, 1024) * 4 * 8, dtype=torch.int32, device=dev)
N.lib().snvrag_tail_stamps(stp.data_ptr())
for _ in range(10):
    tail_var(0, persist=1)()
tail_var(7, persist=1)()
torch.cuda.synchronize()
N.lib().snvrag_tail_stamps(None)
K.set_option("tail_variant", 0)
t = stp[:G * 4 * 8].view(G * 4, 8).cpu().numpy().astype(np.int64) & 0xffffffff
ph = ["tile start (first tile: slab 0 + no-op stores)", "out-projection groups (A_g, W_o', R_g; 288 MFMA)",
      "sync of the first FFN slab", "LN1", "FFN (2304 MFMA)", "LN2 + stores"]
tot = (t[:, 6] - t[:, 0]) % (1 << 32)
print(f"tailp stamped launch: {G} workgroups, last tile of each wave", flush=True)
for i, nm in enumerate(ph):
    d = (t[:, i + 1] - t[:, i]) % (1 << 32)
    print(f"  {nm:40s} median {np.median(d):9.0f} cyc  p10 {np.percentile(d, 10):9.0f}  p90 {np.percentile(d, 90):9.0f}"
          f"  ({np.median(d) / np.median(tot):.3f} of the tile)", flush=True)
print(f"  {'tile total':40s} median {np.median(tot):9.0f} cyc  (MFMA floor 82944)", flush=True)
