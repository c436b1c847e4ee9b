"""The bench's kNN HBM probe in isolation (bench.py knn_hbm_probe): the full-panel scan of the
bench workload (1M haplotypes x 1024 sites, queries copied from panel rows, aligned masks ->
the one-limb reduced scan) at 48 / 96 / 128 queries, split into its loads-only and compute-only
halves (SNVRAG_SCAN_MODE), plus the whole search (pre-pass + scan + merge) at pre-pass sample
divisors SNVRAG_SAMPLE_DIV in KP_DIVS, and the L2-prefetch variants of the scan (SNVRAG_SCAN_PF)."""
import os
import sys
from types import SimpleNamespace

import torch

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [REPO, os.path.join(REPO, "rag-snvbert_amd")]
import bench  # noqa: E402
from src import kernels as K  # noqa: E402
from src.dataset import synthetic  # noqa: E402
from src.dataset.vocab import WordVocab  # noqa: E402


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


dev = torch.device("cuda")
args = SimpleNamespace(batch=64, n_ref=1_000_000, window=1024, level=4)
wl = bench.build_workload(args, dev, WordVocab(synthetic.POPS))
W = torch.randn(12, 384, device=dev)
ix = wl.index
byts = ix.n_ref * ix.n_sites_pad
for nq in [int(v) for v in os.environ.get("KP_NQ", "48,96,128").split(",")]:
    tq = wl.tok[:nq].contiguous()
    lut, exps, consts = ix.lut(tq, W, wl.site_mask, 2)
    keys = ix.scan_keys(lut, nq, 2, 32)
    th = K.knn_threshold(keys, 32)
    # the threshold a 1/128 pre-pass gives (the r2 default)
    m = max(16 * 32, ((ix.n_ref // 128) + 15) // 16 * 16)
    th128 = K.knn_threshold(K.topk_merge(K.knn_scan(ix.codes[:m], ix.n_sites_pad, lut, nq, 2, 32, 0,
                                                    n_parts=max(1, min(256, m // 64))), 32), 32)
    for mode, name in (("0", "full"), ("1", "loads only"), ("2", "compute only")):
        K.set_option("scan_mode", int(mode))
        for tname, t in (("th1/128", th128), ("th exact", th)):
            ms = timeit(lambda: K.knn_scan(ix.codes, ix.n_sites_pad, lut, nq, 2, 32, 0, th_init=t))
            print(f"nq={nq:3d} scan {name:12s} {tname:8s}: {ms:7.4f} ms {byts / ms / 1e6:8.1f} GB/s "
                  f"({byts / ms / 1e6 / 8000:.3f} of 8 TB/s)", flush=True)
    K.set_option("scan_mode", 0)
    for div in os.environ.get("KP_DIVS", "128,64,32").split(","):
        os.environ["SNVRAG_SAMPLE_DIV"] = div
        ms = timeit(lambda: ix.scan_keys(lut, nq, 2, 32))
        print(f"nq={nq:3d} search (pre-pass 1/{div} + scan + merge): {ms:7.4f} ms", flush=True)
    os.environ.pop("SNVRAG_SAMPLE_DIV", None)
