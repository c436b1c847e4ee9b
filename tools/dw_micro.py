"""Linear weight-gradient kernel (csrc/dw.hip) at the training shapes (M = 2 * 24 * 1030 rows):
time per launch for several M-split counts (the split count sets the number of workgroups and
of f32 atomic adds: splits * N * K), TFLOP/s."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
from src import kernels as K  # noqa: E402
from src import native as N  # noqa: E402

M = int(os.environ.get("M", 2 * 24 * 1030))
shapes = [(384, 1536), (1536, 384), (1152, 384), (384, 384)]
torch.manual_seed(0)
ROT = int(os.environ.get("ROT", 3))
XCD = [int(v) for v in os.environ.get("DW_XCD", "1").split(",")]
for xcd, (n, k) in [(v, sh) for sh in shapes for v in XCD]:
    K.set_option("dw_xcd", xcd)
    # ROT operand copies used in turn (3 x 190 MB at the FFN shapes > the 256 MB MALL: every
    # launch reads its operands from HBM, as in the training step)
    dys = [(torch.randn(M, n, device="cuda") * 0.1).to(torch.bfloat16) for _ in range(ROT)]
    xs = [torch.randn(M, k, device="cuda").to(torch.bfloat16) for _ in range(ROT)]
    dw = torch.zeros(n, k, device="cuda")
    tiles = (n // 128) * (k // 128)
    dflt = N.lib().snvrag_dw_splits(M, n, k)
    res = []
    for s in sorted({dflt, max(1, 256 // tiles), max(1, 512 // tiles), max(1, 128 // tiles), 2 * dflt}):
        K.linear_dw(dys[0], xs[0], splits=s, dw=dw)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(21):
            K.linear_dw(dys[i % ROT], xs[i % ROT], splits=s, dw=dw)
        b.record()
        torch.cuda.synchronize()
        ms = a.elapsed_time(b) / 21
        res.append(f"s={s}{'*' if s == dflt else ''}: {ms * 1e3:.1f} us {2 * M * n * k / ms / 1e9:.0f} TF/s")
    print(f"N={n} K={k} tiles={tiles} xcd={xcd}: " + "  ".join(res), flush=True)
