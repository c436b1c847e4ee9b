"""The 4-wave stream-GEMM launches (and with OPT=mlp_desync the MLP kernels) (emb_fusion LN, the rag fusion's cat GEMM, the hap head's
net[0] + head epilogue) at the bench shapes vs the first-round stagger (option sg_desync; -1 = the
launcher default, 0 for 4-wave launches), interleaved repeats, HIP events."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd"))
sys.path.insert(0, os.path.dirname(__file__))
import sg_family_micro as S  # noqa: E402  (builds the operands at the bench shapes)
from src import kernels as K  # noqa: E402

cases = [c for c in S.cases if c[0] in os.environ.get("CASES", "cat GEMM,head net0+head2,emb_fusion LN").split(",")]
vals = [int(v) for v in os.environ.get("DZ", "-1,5000,10000,20000,40000").split(",")]


OPT = os.environ.get("OPT", "sg_desync")


def timeit(fn, dz, reps=10):
    K.set_option(OPT, dz)
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for name, fn, fl in cases:
    res = {v: [] for v in vals}
    for _ in range(int(os.environ.get("REPS", 5))):
        for v in vals:
            res[v].append(timeit(fn, v))
    print(name, "  ".join(f"{v}: {sorted(res[v])[len(res[v]) // 2]:.4f}" for v in vals), flush=True)
K.set_option(OPT, -1)
