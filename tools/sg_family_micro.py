"""Launch times of the stream-GEMM family (csrc/sgemm.hip) at the bench shapes (B = 256, L = 1030,
D = 384): QKV (8 waves), the rag fusion's cat GEMM, the hap head's net[0] + head epilogue, the
emb_fusion LN form, the hap head's af_fusion MLP and the AF-gate MLP.  HIP events, median of
5 x 10 launches; run once per library build (SNVRAG_LIB) to A/B compile-time variants."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402
from src import native as N  # noqa: E402

D, H = 384, 1536
BL = 256 * 1030
M2 = 2 * BL
dev, bf = "cuda", torch.bfloat16
g = torch.Generator(device="cpu").manual_seed(0)
rn = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).to(dev)
wq = (rn(3 * D, D) / math.sqrt(D)).to(bf)
w4 = (rn(H, D) / math.sqrt(D)).to(bf)
wc = (rn(H, 2 * D) / math.sqrt(2 * D)).to(bf)
w2 = (rn(D, H) / math.sqrt(H)).to(bf)
wd = (rn(D, D) / math.sqrt(D)).to(bf)
x2 = rn(M2, D).to(bf)
x4 = rn(2 * M2, D).to(bf)
xr = rn(M2, D).to(bf)
aw = torch.rand(BL, D, generator=g).to(dev, bf)
af, afp = torch.rand(BL, generator=g).to(dev), torch.rand(BL, generator=g).to(dev)
pf = torch.rand(BL, generator=g).to(dev)

qkv_s, qkv_v = K.sgemm_pack(wq), K.sgemm_vec(rn(3 * D))
cat_s, cat_v = K.sgemm_pack(wc), K.sgemm_vec(rn(H))
hd_s = K.sgemm_pack(w4)
hd_v = K.sgemm_vec(rn(H), head=(rn(2, H, sc=0.03), rn(2)))
ef_s = K.sgemm_pack(wd)
ef_v = K.sgemm_vec(rn(D), rn(D), rn(D), ln=(1 + rn(D, sc=0.1), rn(D, sc=0.1)))
ml_s = K.mlp_pack(w4, w2)
ml_v = torch.cat([rn(H), rn(H), rn(H), rn(D), 1 + rn(D, sc=0.1), rn(D, sc=0.1)]).contiguous()
ag = [rn(32, 2, sc=0.8), rn(32, sc=0.1), rn(D, 32, sc=0.25), rn(D, sc=0.1), rn(D, 2, sc=0.7), rn(D, sc=0.1),
      1 + rn(D, sc=0.1), rn(D, sc=0.1)]
afg_f, afg_v = K.mlp_afgate_pack(ag, torch.cat([rn(H), rn(D, sc=0.1)]).contiguous())


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(e) / reps)
    return sorted(ts)[2]


cases = [
    ("QKV 8 waves", lambda: K.sgemm(x2, qkv_s, 3 * D, qkv_v), 2.0 * M2 * D * 3 * D),
    ("cat GEMM", lambda: K.sgemm_cat(x2, xr, aw, BL, cat_s, H, cat_v), 2.0 * M2 * 2 * D * H),
    ("head net0+head2", lambda: K.sgemm(x2, hd_s, H, hd_v, epi=K.SG_HEAD2, act=N.ACT_GELU), 2.0 * M2 * D * H),
    ("emb_fusion LN", lambda: K.sgemm(x4, ef_s, D, ef_v, epi=K.SG_LN, act=N.ACT_LRELU, slope=0.1, rank=(pf, af, BL)),
     2.0 * 2 * M2 * D * D),
    ("af_fusion MLP", lambda: K.mlp(x2, ml_s, ml_v, epi2=1, rank=(af, afp, BL)), 4.0 * M2 * D * H),
    ("AF-gate MLP", lambda: K.mlp_afgate(af, afp, afg_f, 0.1, ml_s, afg_v), 4.0 * BL * D * H),
]
if __name__ == "__main__":
    print(f"library {N.LIB_PATH}", flush=True)
    tot = 0.0
    for name, fn, fl in cases:
        t = timeit(fn)
        tot += t
        print(f"{name:18s} {t:.4f} ms  {fl / t / 1e9 / 2500:.3f} of 2.5 PF", flush=True)
    print(f"sum (QKV x12 counted once) {tot:.4f} ms", flush=True)
