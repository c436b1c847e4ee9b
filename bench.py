"""Benchmark of the v18 embedding-RAG imputation hot path on MI355X.

One step = one batch of B synthetic samples (2B query haplotypes) through:
  retrieval: LUT -> int8-MFMA scan of the HBM-resident panel (N haplotypes x
             window sites) -> exact top-k merge -> neighbour K-mean (rag_mean)
  forward:   embedding + emb_fusion + rag_fusion + 12-block encoder + heads
             (BERTFoundationModel eval forward, bf16 compute, f32 accumulation)
Metric (BASELINE.json): masked SNVs imputed/s (2 * sum(mask) per sample-window),
with kNN queries/s reported beside it.  Workload = configs[2] of BASELINE.json:
window 1024 sites, k = 32, 1M-haplotype panel resident in HBM, d384/L12/H12.

Launch: python bench.py --gpus N --steps K --warmup W.  N>1 runs one rank per GPU: under
torch.distributed.run (WORLD_SIZE set) this process is one rank and checks WORLD_SIZE == N;
started directly, it first checks that N devices are visible (exit 2 otherwise) and then
starts ``torch.distributed.run --nproc-per-node N`` on itself as a child process before any
GPU call, exiting with the child's status.  Each rank imputes its own B samples -> weak scaling.  With N>1 the
default ``--panel sharded`` gives every rank a contiguous 1/N of the panel: the search
all-gathers the ranks' query tokens, scans the local shard, all-gathers and merges the
partial top-k keys and all-reduces the neighbours' alt-allele counts over RCCL
(src/retrieval/shards.py); ``--panel replicated`` keeps a full HBM copy per
rank and runs no data-path collective.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "rag-snvbert_amd"))

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
BF16_PEAK_TFLOPS = 2500.0    # dense bf16 MFMA (no sparsity)
F32_PEAK_TFLOPS = 157.3


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="ranks = GPUs (default: WORLD_SIZE under a launcher, else 1)")
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--batch", type=int, default=256,
                   help="samples per step per GPU (configs[4]'s inference batch; 512 haplotype sequences)")
    p.add_argument("--n-ref", type=int, default=1_000_000, help="panel haplotypes")
    p.add_argument("--window", type=int, default=1024, help="sites per window")
    p.add_argument("--k", type=int, default=32)
    p.add_argument("--dims", type=int, default=384)
    p.add_argument("--layers", type=int, default=12)
    p.add_argument("--heads", type=int, default=12)
    p.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    p.add_argument("--level", type=int, default=4, help="curriculum mask level (dataset.py:252 rates [0.3 .. 0.8]: 4 -> 70%%; "
                        "sites with AF < 0.05 always 70%%)")
    p.add_argument("--f32-leg", type=int, default=2,
                   help="steps of the same batch on the exact-f32 path (bf16-vs-f32 call agreement); 0 = skip")
    p.add_argument("--cpu-baseline", type=int, default=1, help="time the oracle on host cores (rank 0)")
    p.add_argument("--cpu-panel", type=int, default=65536, help="panel sample for the CPU kNN timing")
    p.add_argument("--panel", default="sharded", choices=["sharded", "replicated"],
                   help="N>1: each rank holds 1/N of the panel and serves every rank's queries (SURVEY §8e), "
                        "or every rank holds the whole panel")
    p.add_argument("--c2-n", type=int, default=10_000,
                   help="SURVEY §8d C2 embedding-space cross-check: panel haplotypes embedded (bf16 [N, 1030*D]); 0 = skip")
    p.add_argument("--train-steps", type=int, default=3,
                   help="timed DDP training steps at configs[1] (B=24/GPU, window 512, k=8, 10k-haplotype panel); 0 = skip")
    p.add_argument("--train-window", type=int, default=512, help="configs[1] window (sites) of the training leg")
    p.add_argument("--one-device-rehearsal", action="store_true",
                   help="N>1 rehearsal on a one-GPU box: every rank on cuda:0 over gloo (host-staged "
                        "collectives); the numbers are not a measurement")
    return p.parse_args(argv)


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(args, argv, port):
    """The torch.distributed.run command that starts ``args.gpus`` ranks of this script."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve()), *argv]


def check_devices(n_ranks: int, n_devices: int, rehearsal: bool) -> None:
    """Exit (status 2, message on stderr) instead of measuring fewer GPUs than asked for."""
    if not rehearsal and n_devices < n_ranks:
        sys.stderr.write(f"bench.py: --gpus {n_ranks} needs {n_ranks} visible GPUs, found {n_devices}; "
                         "not measuring (no n_gpus line is printed)\n")
        sys.exit(2)


def launch_ranks(args, argv) -> int:
    """--gpus N > 1 without a launcher: start N ranks (one per GPU) as a CHILD process — this
    process has not touched the GPU (torch.cuda.device_count() does not initialise it) and
    does not exec; its exit status is the launcher's."""
    import subprocess
    check_devices(args.gpus, torch.cuda.device_count(), args.one_device_rehearsal)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(launch_command(args, argv, _free_port()), env=env)


def setup_dist(args):
    """This rank's (world, rank, local device).  The world must be the --gpus asked for, and
    every rank needs its own visible GPU (RCCL: one process per GPU); the rehearsal puts every
    rank on cuda:0 over gloo."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        sys.stderr.write(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks\n")
        sys.exit(2)
    args.gpus = world
    check_devices(world, torch.cuda.device_count(), args.one_device_rehearsal)
    dev_i = 0 if args.one_device_rehearsal else local
    torch.cuda.set_device(dev_i)
    if world > 1:
        import torch.distributed as dist
        if args.one_device_rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{dev_i}"))
        assert dist.get_world_size() == world == args.gpus, (dist.get_world_size(), world, args.gpus)
    return world, rank, dev_i


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def dist_info(world):
    """The collective backend this run measured on (the bench line's ``distributed``)."""
    if world <= 1:
        return {"backend": None, "world_size": 1}
    import torch.distributed as dist
    be = dist.get_backend()
    return {"backend": "rccl" if be == "nccl" else be, "world_size": dist.get_world_size(),
            "rehearsal_one_device": be == "gloo"}


def max_over_ranks(v: float, world: int, dev) -> float:
    """MAX of a host float over the ranks (gloo: through a host tensor)."""
    if world <= 1:
        return v
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64, device=dev if dist.get_backend() != "gloo" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def make_queries(args, af_np, seed, rank):
    """B samples whose haplotypes copy panel rows (hash-generated like the device panel) with 2% flips."""
    from src.dataset.synthetic import hash_uniform
    rng = np.random.default_rng([seed, rank])
    B, S = args.batch, args.window
    src = rng.integers(0, args.n_ref, size=(B, 2))
    cols = np.arange(S)
    alle = (hash_uniform(seed, src[..., None], cols[None, None]) < af_np[None, None]).astype(np.uint8)
    alle ^= (rng.random(alle.shape) < 0.02).astype(np.uint8)
    return alle, src


def build_workload(args, dev, vocab, rank=0, seed=1234, shard=None):
    """configs[2] workload: one window of ``args.window`` sites, an ``args.n_ref``-haplotype panel
    generated on the device (HBM-resident; with ``shard`` only this rank's contiguous range of
    it), ``args.batch`` query samples copied from panel rows with 2 % flips, AF-guided masks at
    ``args.level``.  Shared by the bench and the launch-shape kNN parity test
    (tests/test_gpu_knn_scale.py)."""
    from types import SimpleNamespace
    from src import kernels as K
    from src.dataset import utils as U
    from src.retrieval import PanelIndex
    S, B, L = args.window, args.batch, 1030
    rng = np.random.default_rng(seed)
    af_np = rng.beta(0.3, 3.0, S).astype(np.float32)
    pos = np.sort(rng.choice(np.arange(1, 50 * S), S, replace=False))
    af_dev = torch.from_numpy(af_np).to(dev)
    ref_af = U.sequence_padding(af_np, "float").astype(np.float32)
    if shard is None:
        index = PanelIndex.synthetic(args.n_ref, S, af_dev, torch.from_numpy(ref_af).to(dev), seed)
    else:
        r0, r1 = shard.bounds(args.n_ref)
        index = PanelIndex(K.panel_synth(r1 - r0, S, af_dev, seed, row0=r0), S, torch.from_numpy(ref_af).to(dev),
                           ref_offset=r0, n_total=args.n_ref)
    raw_mask = U.af_guided_mask(af_np, args.level, 0, 0)
    mask = U.sequence_padding(raw_mask, "int")
    alle, src = make_queries(args, af_np, seed, rank)
    pad = lambda a: torch.from_numpy(np.stack([U.sequence_padding(r, "float") for r in a]).astype(np.float32)).to(dev)
    afp = np.clip(af_np[None] + 0.05 * rng.standard_normal((B, S)), 0, 1)
    x = dict(hap_1=torch.from_numpy(vocab.tokenize(alle[:, 0], mask)).to(dev),
             hap_2=torch.from_numpy(vocab.tokenize(alle[:, 1], mask)).to(dev),
             af=pad(np.broadcast_to(af_np, (B, S))), af_p=pad(afp),
             pos=pad(np.broadcast_to(U.position_normalize(pos), (B, S))),
             ref=pad((1 - afp) ** 2), het=pad(2 * afp * (1 - afp)), hom=pad(afp ** 2))
    site_mask = torch.from_numpy(raw_mask.astype(np.uint8)).to(dev)
    tok = torch.cat([x["hap_1"], x["hap_2"]]).contiguous()
    return SimpleNamespace(index=index, x=x, site_mask=site_mask, tok=tok, raw_mask=raw_mask, af_np=af_np,
                           ref_af=ref_af, alle=alle, src=src, S=S, B=B, L=L, shard=shard,
                           masked_per_step=2 * B * int(raw_mask.sum()))


def make_search(wl, eng, k):
    """The exact kNN of the step's 2B query haplotypes -> (idx [2B, k], counts or None).
    Sharded panel: the collective search of src/retrieval/shards.py (every rank's queries
    against every shard; the neighbours' alt-allele counts come back all-reduced)."""
    P = eng.packed()
    if wl.shard is None:
        return lambda: (wl.index.search(wl.tok, P.W, wl.site_mask, k)[0], None)
    from src.retrieval.shards import kernel_ops, sharded_neighbours
    ops = kernel_ops(wl.index, P.W, wl.site_mask, k)

    def search():
        idx, _, counts = sharded_neighbours(wl.tok, k, ops, None, wl.shard.group)
        return idx, counts
    return search


def make_step(wl, eng, k):
    """One step: exact kNN over the panel -> neighbour K-mean written straight into the
    encoder's input block -> full eval forward (engine dtype)."""
    from src import kernels as K
    P = eng.packed()
    Ar = eng.af_embedding(torch.from_numpy(wl.ref_af).to(wl.tok.device)[None]).float()[0].contiguous()
    B, L, D = wl.B, wl.L, P.D
    search = make_search(wl, eng, k)

    def step():
        idx, counts = search()
        block = torch.empty(4 * B, L, D, device=wl.tok.device, dtype=eng.dtype)
        K.rag_mean(idx, wl.index.codes, wl.S, P.W, P.pe, Ar, L, eng.dtype, out=block[2 * B:], counts=counts)
        wl.x["rag_block"] = block
        return eng.forward(wl.x)
    return step


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, argv))
    world, rank, local = setup_dist(args)
    dev = torch.device(f"cuda:{local}")
    from src import native as N
    from src.dataset import synthetic
    from src.dataset.vocab import WordVocab
    from src.engine import engine_for
    from src.model import build_model

    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    vocab = WordVocab(synthetic.POPS)
    torch.manual_seed(0)
    model = build_model(len(vocab), args.dims, args.layers, args.heads).to(dev).eval()
    eng = engine_for(model)
    eng.set_dtype(dtype)
    P = eng.packed()

    # ---- window, panel (HBM-resident, generated on device), queries ----
    shard = None
    if world > 1 and args.panel == "sharded":
        from src.retrieval.shards import PanelShard
        shard = PanelShard.current()
    wl = build_workload(args, dev, vocab, rank, shard=shard)
    S, B, L = wl.S, wl.B, wl.L
    index, x, tok, site_mask = wl.index, wl.x, wl.tok, wl.site_mask
    af_np, ref_af, raw_mask = wl.af_np, wl.ref_af, wl.raw_mask
    masked_per_step = wl.masked_per_step
    index_sites_pad = index.n_sites_pad
    k = args.k
    step = make_step(wl, eng, k)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    lib = N.lib()
    cap = 4096
    lib.snvrag_evlog_enable(cap)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    barrier(world)
    elapsed = time.perf_counter() - t0
    kinds = np.zeros(cap, np.int32)
    ms = np.zeros(cap, np.float32)
    work = np.zeros(cap, np.float64)
    n = lib.snvrag_evlog_read(kinds.ctypes.data, ms.ctypes.data, work.ctypes.data, cap)
    lib.snvrag_evlog_enable(0)
    kinds, ms, work = kinds[:n], ms[:n], work[:n]
    # the whole kNN search (LUT + pre-pass + scan + merges + decode) alone, outside the timed region
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    search = make_search(wl, eng, k)
    ev0.record()
    for _ in range(5):
        search()
    ev1.record()
    torch.cuda.synchronize()
    knn_ms = ev0.elapsed_time(ev1) / 5
    # HBM-regime probes (SURVEY.md §8d states the HBM target at Bq in {48, 96}): the scan
    # streams the panel once per launch; up to ~150 queries the int8 MFMA work per code
    # byte is below the HBM ridge
    probes = []
    for nq in (48, 96, 128):
        tq = tok[:nq].contiguous()
        index.search(tq, P.W, site_mask, k)
        lib.snvrag_evlog_enable(cap)
        for _ in range(5):
            index.search(tq, P.W, site_mask, k)
        torch.cuda.synchronize()
        kk, mm, ww = np.zeros(cap, np.int32), np.zeros(cap, np.float32), np.zeros(cap, np.float64)
        n2 = lib.snvrag_evlog_read(kk.ctypes.data, mm.ctypes.data, ww.ctypes.data, cap)
        lib.snvrag_evlog_enable(0)
        kk, mm, ww = kk[:n2], mm[:n2], ww[:n2]
        sel = (kk == 4) & (ww >= 0.5 * ww[kk == 4].max())
        pr = dict(queries=nq, avg_launch_ms=round(float(mm[sel].mean()), 4),
                  bytes_per_launch=float(ww[sel].mean()),
                  achieved_gbs=round(float(ww[sel].sum() / (mm[sel].sum() * 1e-3)) / 1e9, 1))
        pr["frac"] = round(pr["achieved_gbs"] / HBM_PEAK_GBS, 4)
        probes.append(pr)
    probe = dict(probes[-1], per_queries=[{kq: p[kq] for kq in ("queries", "avg_launch_ms", "achieved_gbs", "frac")}
                                          for p in probes])
    c2 = knn_c2(args, wl, eng, k) if (args.c2_n > 0 and rank == 0 and dtype == torch.bfloat16) else None
    # precision leg: the same batch through the exact-f32 path, whose logits
    # carry the 1e-3 parity bar; report how often the bf16 run's imputed calls agree with it
    precision = precision_leg(args, wl, eng, k, out) if (args.f32_leg and dtype == torch.bfloat16) else None
    elapsed = max_over_ranks(elapsed, world, dev)

    def agg(kind):
        sel = kinds == kind
        cnt = int(sel.sum())
        if cnt == 0:
            return None
        return dict(launches_per_step=cnt / args.steps, avg_ms=float(ms[sel].mean()),
                    work_per_launch=float(work[sel].mean()), total_ms_per_step=float(ms[sel].sum()) / args.steps,
                    rate=float(work[sel].sum() / (ms[sel].sum() * 1e-3)))

    gemm, attn, ln, ffn = agg(1), agg(2), agg(3), agg(8)
    # kNN: the full-panel scan launch (the threshold pre-pass over a 1/64 prefix is
    # reported with the rest of the search path)
    full = (kinds == 4) & (work >= 0.5 * work[kinds == 4].max())
    kinds = np.where((kinds == 4) & ~full, 9, kinds)
    scan, prescan = agg(4), agg(9)
    ms_step = elapsed / args.steps * 1e3
    value = masked_per_step * world * args.steps / elapsed
    knn_qps = 2 * B * world * args.steps / elapsed
    del index, out
    torch.cuda.empty_cache()
    train = train_bench(args, world, rank, dev) if args.train_steps > 0 else None
    if rank != 0:
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    peak_f = BF16_PEAK_TFLOPS if dtype == torch.bfloat16 else F32_PEAK_TFLOPS
    # roofline object = the MFMA kernel class with the most time per step
    mf = [("rows_gemm_kernel (encoder QKV/out-proj + fusion/head GEMMs)", gemm, "2*M*N*K averaged over launches"),
          ("tailw_kernel (wide-row block tail on 32x32 MFMAs: out-projection + LN1 + FFN + LN2, 12 launches)", ffn,
           "2*M*D*9D = 18*M*D^2 per launch"),
          ("attn32_dma (attention)", attn, "4*L^2*dh*H*nseq per launch")]
    name, dom, per = max((m for m in mf if m[1]), key=lambda m: m[1]["total_ms_per_step"])
    tr = pmc_traffic(name)
    roofline = dict(bound="mfma", kernel=name,
                    achieved=round(dom["rate"] / 1e12, 2), peak=peak_f, unit="TFLOP/s",
                    frac=round(dom["rate"] / 1e12 / peak_f, 4),
                    traffic=tr["bytes_per_launch"] if tr else None, traffic_unit="HBM bytes per launch",
                    traffic_detail=tr,
                    avg_launch_ms=round(dom["avg_ms"], 4),
                    algorithmic_per_launch=f"{dom['work_per_launch']:.4g} FLOP ({per})")
    extra = {
        "kernels": {
            "attention": dict(achieved_tflops=round(attn["rate"] / 1e12, 2), frac=round(attn["rate"] / 1e12 / peak_f, 4),
                              ms_per_step=round(attn["total_ms_per_step"], 3)),
            "knn_scan": dict(queries=2 * B, achieved_gbs=round(scan["rate"] / 1e9, 1), peak=HBM_PEAK_GBS,
                             frac_hbm=round(scan["rate"] / 1e9 / HBM_PEAK_GBS, 4),
                             int8_tops=round(2.0 * 2 * B * args.n_ref * index_sites_pad / (scan["avg_ms"] * 1e-3) / 1e12, 1),
                             avg_launch_ms=round(scan["avg_ms"], 4), bytes_per_launch=scan["work_per_launch"],
                             prepass_ms=round(prescan["total_ms_per_step"], 4) if prescan else 0.0,
                             note="all queries in one pass over the panel (XCD co-scheduled query groups); "
                                  "above ~150 queries the scan is int8-MFMA/LDS bound, see knn_hbm_probe"),
            "knn_hbm_probe": dict(probe, bound="hbm", peak=HBM_PEAK_GBS),
            "knn_c2_embedding_space": c2,
            "knn_search_ms": round(knn_ms, 4),
            # (sharded panel: the search serves every rank's queries in that time)
            "knn_search_queries_per_s": round(2 * B * (world if shard is not None else 1) / (knn_ms * 1e-3), 1),
            "gemm": dict(achieved_tflops=round(gemm["rate"] / 1e12, 2), frac=round(gemm["rate"] / 1e12 / peak_f, 4),
                         ms_per_step=round(gemm["total_ms_per_step"], 3), launches_per_step=gemm["launches_per_step"]),
            "ffn_fused": (dict(achieved_tflops=round(ffn["rate"] / 1e12, 2), frac=round(ffn["rate"] / 1e12 / peak_f, 4),
                               ms_per_step=round(ffn["total_ms_per_step"], 3), avg_launch_ms=round(ffn["avg_ms"], 4))
                          if ffn else None),
            "layernorm": (dict(ms_per_step=round(ln["total_ms_per_step"], 3), achieved_gbs=round(ln["rate"] / 1e9, 1))
                          if ln else "fused into GEMM epilogues/prologues"),
        },
        "knn_queries_per_s": round(knn_qps, 1),
        "masked_snvs_per_step_per_gpu": masked_per_step,
    }
    from src.dataset import utils as U
    cpu = None
    if args.cpu_baseline and world == 1:             # rank 0 at N = 1 only (the other ranks would idle)
        cpu = cpu_baseline(args, model, vocab, af_np, ref_af, raw_mask, x, dev)
    line = {
        "metric": "masked SNVs imputed/sec (+ kNN queries/sec), window=1024 k=32",
        "value": round(value, 1), "unit": "masked SNVs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (seeded AF~Beta(0.3,3) panel + copied queries)",
        "config": {"workload": "configs[2]: v18 embedding-RAG imputation, window=1024 sites (L=1030 tokens), "
                               f"k={k}, {args.n_ref}-haplotype panel resident in HBM, d{args.dims}/L{args.layers}/H{args.heads}",
                   "mask_level": args.level, "mask_rate": U.MASK_RATES[args.level], "rare_mask_rate": 0.7,
                   "masked_site_fraction": round(float(raw_mask.mean()), 4),
                   "global_batch": B * world, "seq_len": L, "parallelism": (f"dp{world} + panel sharded {world}-way" if shard is not None
                                                  else f"dp{world} (panel replicated)")},
        "roofline": roofline, "cpu_baseline": cpu, **extra, "precision_parity": precision, "train": train,
        "distributed": dist_info(world),
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def call_agreement(o_lo, o_hi, raw_mask):
    """Imputed-call agreement of two forwards over the masked sites (token l = site + 1):
    haplotype calls p(alt) > 0.5 (infer_embedding_rag.py:145-152: softmax is monotone, so the
    reference's second softmax does not move the threshold) and the genotype argmax."""
    sites = torch.from_numpy(np.nonzero(raw_mask)[0] + 1).to(o_lo["probs_h1"].device)
    hp = lambda o: torch.stack([o["probs_h1"][:, sites, 1], o["probs_h2"][:, sites, 1]]).float()
    a, b = hp(o_lo), hp(o_hi)
    ga, gb = o_lo["gt"][:, sites].argmax(-1), o_hi["gt"][:, sites].argmax(-1)
    margin = (b - 0.5).abs()
    conf = margin > 2e-2                     # f32 call clear of the bf16 probability tolerance
    return dict(masked_haplotype_calls=int(a.numel()),
                hap_call_agreement=round(float(((a > 0.5) == (b > 0.5)).float().mean()), 6),
                hap_call_agreement_confident=round(float(((a > 0.5) == (b > 0.5))[conf].float().mean()), 6)
                if bool(conf.any()) else None,
                confident_fraction=round(float(conf.float().mean()), 4),
                gt_argmax_agreement=round(float((ga == gb).float().mean()), 6),
                max_abs_prob_diff=round(float((a - b).abs().max()), 5),
                mean_abs_prob_diff=round(float((a - b).abs().mean()), 6))


def precision_leg(args, wl, eng, k, out_bf16):
    """Same batch, same neighbours on the exact-f32 engine (f32 MFMA, the 1e-3 logit-parity path):
    its throughput and the bf16 run's call agreement with it."""
    keep = {kk: out_bf16[kk].clone() for kk in ("probs_h1", "probs_h2", "gt")}
    eng.set_dtype(torch.float32)
    step32 = make_step(wl, eng, k)
    out32 = step32()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.f32_leg):
        out32 = step32()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / args.f32_leg
    res = dict(call_agreement(keep, out32, wl.raw_mask), f32_ms_per_step=round(el * 1e3, 2),
               f32_masked_snvs_per_s=round(wl.masked_per_step / el, 1), f32_steps=args.f32_leg)
    eng.set_dtype(torch.bfloat16)
    wl.x.pop("rag_block", None)
    return res


class _TrainFlops:
    """Algorithmic FLOP of one training step, counted from the shapes the train graph hands its
    MFMA nodes (src/train_forward.py): every Linear 6·M·K·N (forward, dX, dW), attention
    12·L²·dh per head and sequence (forward QKᵀ + PV, backward dV, dP, dQ, dK — the backward's
    recomputation of QKᵀ not counted).  The small torch layers (AF gate MLP, Conv1d, the 4-class
    head projection) are left out, so the count is a lower bound."""
    RULE = "6*M*K*N per Linear + 12*L^2*dh*heads*nseq per attention; recompute and small torch layers excluded"

    def __enter__(self):
        from src import train_forward as tf
        self.tf, self.flops = tf, 0
        self.saved = (tf.hip_linear, tf.hip_linear_rank2, tf.hip_attention)

        def lin(x, weight, bias=None, **kw):
            n = sum(w.shape[0] for w in weight) if isinstance(weight, (list, tuple)) else weight.shape[0]
            self.flops += 6 * (x.numel() // x.shape[-1]) * x.shape[-1] * n
            return self.saved[0](x, weight, bias, **kw)

        def lin2(x, ln, c1, c2):
            self.flops += 6 * (x.numel() // x.shape[-1]) * ln.weight.shape[1] * ln.weight.shape[0]
            return self.saved[1](x, ln, c1, c2)

        def att(qkv, nseq, L, heads, dh, *a, **kw):
            self.flops += 12 * L * L * dh * heads * nseq
            return self.saved[2](qkv, nseq, L, heads, dh, *a, **kw)
        tf.hip_linear, tf.hip_linear_rank2, tf.hip_attention = lin, lin2, att
        return self

    def __exit__(self, *exc):
        self.tf.hip_linear, self.tf.hip_linear_rank2, self.tf.hip_attention = self.saved
        return False


def train_bench(args, world, rank, dev):
    """Training throughput at configs[1] / configs[3] shape: per GPU B=24 samples, window 512
    sites (configs[1]; the encoder still runs L = 1030 tokens), k=8 neighbours from a
    10k-haplotype panel, d384/L12/H12, bf16 + f32 master weights.
    One step = retrieval + forward + focal losses + backward + bucketed all-reduce (RCCL when
    world > 1) + clipped fused Adam.  Timed like the main metric (barrier + sync around).
    With world > 1 every rank builds the SAME panel and global batch and trains on its own 24
    samples; ``--panel sharded`` (configs[3]) gives each rank a contiguous 1/world of the panel
    and the retrieval runs the collective search (src/retrieval/shards.py)."""
    from src.dataset.embedding_rag_dataset import embedding_rag_collate_fn
    from src.dataset.synthetic import make_rag_dataset
    from src.main.pretrain_with_val_optimized import BERTTrainerWithValidationOptimized
    from src.model import build_model
    Bt, S, nref = 24, args.train_window, 5000
    # the epoch-0 window masks come from numpy's global RNG (the reference's semantics; its CLI
    # seeds it first): seeded here so every run and every rank retrieves from the same masks
    np.random.seed(7)
    ds, vocab = make_rag_dataset(n_samples=Bt * world, n_sites=S, n_windows=1, n_ref_samples=nref, seed=7,
                                 name="train")
    shard = None
    if world > 1 and args.panel == "sharded":
        from src.retrieval.shards import PanelShard
        shard = PanelShard.current()
        ds.set_panel_shard(shard)
    batch = embedding_rag_collate_fn([ds[i] for i in range(rank * Bt, (rank + 1) * Bt)])
    torch.manual_seed(0)
    model = build_model(len(vocab), args.dims, args.layers, args.heads).to(dev)
    if world > 1:
        import torch.distributed as dist
        gloo = dist.get_backend() == "gloo"
        for t in list(model.parameters()) + list(model.buffers()):
            if gloo:
                h = t.data.cpu()
                dist.broadcast(h, 0)
                t.data.copy_(h)
            else:
                dist.broadcast(t.data, 0)
    tr = BERTTrainerWithValidationOptimized(model, None, None, vocab, lr=7.5e-5, warmup_steps=100,
                                            grad_accum_steps=1, log_freq=0)
    tr.rag_train_dataset = ds
    tr.rag_k = 8
    for _ in range(2):
        loss = tr.train_step(dict(batch))
    with _TrainFlops() as fl:                     # one more warm-up step, its GEMM shapes counted
        loss = tr.train_step(dict(batch))
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.train_steps):
        loss = tr.train_step(dict(batch))
    torch.cuda.synchronize()
    barrier(world)
    el = max_over_ranks(time.perf_counter() - t0, world, dev)
    masked = 2 * int(batch["mask"].sum())
    ms = el / args.train_steps * 1e3
    tflops = fl.flops / (ms * 1e-3) / 1e12
    return {"ms_per_step": round(ms, 2), "samples_per_s": round(Bt * world * args.train_steps / el, 1),
            "algorithmic_tflop_per_step": round(fl.flops / 1e12, 3), "achieved_tflops": round(tflops, 1),
            "frac_bf16_peak": round(tflops / BF16_PEAK_TFLOPS, 4), "flop_count": fl.RULE,
            "masked_snvs_per_s": round(masked * world * args.train_steps / el, 1),
            "batch_per_gpu": Bt, "window_sites": S, "k": 8, "panel_haplotypes": 2 * nref,
            "panel": (f"sharded {world}-way" if shard is not None else "replicated"),
            "n_gpus": world, "loss": round(float(loss), 3),
            "note": "DDP: bucketed async all-reduce of the flat f32 gradient buffer over RCCL; "
                    "reference banner: 115 ms/batch at B=24 on an unstated GPU (BASELINE.md)"}


def knn_c2(args, wl, eng, k):
    """SURVEY §8d C2 embedding-space mode (cross-check of the token index): the reference's
    literal retrieval — bf16 window embeddings of the first ``args.c2_n`` panel haplotypes,
    [N, 1030 * D] (stored in the scan's tiled layout), exact L2 + top-k (csrc/knn_emb.hip distance GEMM, HBM-bound) — timed at
    Bq in {48, 96}; its neighbours checked against the token index's exact distances; and the
    reference-equivalent CPU cost (torch.cdist + topk over a panel sample, the v18 training
    path's own call) on the host cores."""
    from src import kernels as K
    from src import native as N
    from src.dataset import utils as U
    from src.retrieval import EmbeddingIndex, PanelIndex, panel_tokens
    P = eng.packed()
    dev = wl.tok.device
    n, L, D, S = min(args.c2_n, wl.index.n_ref), wl.L, P.D, wl.S
    codes = wl.index.codes[:n]
    Ar = eng.af_embedding(torch.from_numpy(wl.ref_af).to(dev)[None]).float()[0].contiguous()
    mask = U.sequence_padding(wl.raw_mask, "int")
    tr = panel_tokens(codes, S, mask, L)
    eidx = EmbeddingIndex.build(tr, P.W, P.pe, Ar)
    lib, cap = N.lib(), 256
    out = dict(mode="embedding-space exact L2 (reference-literal cdist / IndexFlatL2 over bf16 [N, L*D])",
               panel_haplotypes=n, dims=L * D, index_bytes=int(eidx.n * L * D * 2), bound="hbm", peak=HBM_PEAK_GBS,
               per_queries=[])
    for bq in (48, 96):
        Q = eidx.embed_queries(wl.tok[:bq], P.W, P.pe, Ar)
        qn = K.knn_emb_norms(Q)
        K.knn_emb_dist(eidx.Et, Q, eidx.norms, qn)
        lib.snvrag_evlog_enable(cap)
        for _ in range(5):
            K.knn_emb_dist(eidx.Et, Q, eidx.norms, qn)
        torch.cuda.synchronize()
        kk, mm, ww = np.zeros(cap, np.int32), np.zeros(cap, np.float32), np.zeros(cap, np.float64)
        n2 = lib.snvrag_evlog_read(kk.ctypes.data, mm.ctypes.data, ww.ctypes.data, cap)
        lib.snvrag_evlog_enable(0)
        sel = kk[:n2] == 4
        ms, by = float(mm[:n2][sel].mean()), float(ww[:n2][sel].mean())
        gbs = by / (ms * 1e-3) / 1e9
        out["per_queries"].append(dict(queries=bq, avg_launch_ms=round(ms, 4), bytes_per_launch=by,
                                       achieved_gbs=round(gbs, 1), frac=round(gbs / HBM_PEAK_GBS, 4)))
    # cross-check at Bq = 96 against the token index over the same sub-panel: exact distances
    # (float64 sums of ||W[a] - W[b]||^2 over token positions) of both neighbour lists
    d_e, idx_e = eidx.search(Q, k)
    pidx = PanelIndex(codes, S, wl.index.ref_af)
    idx_t, _ = pidx.search(wl.tok[:96], P.W, wl.site_mask, k)
    W64 = P.W.double()
    T = ((W64[:, None] - W64[None]) ** 2).sum(-1)
    tq = wl.tok[:96]

    def exact(ix):
        tr_sel = tr[ix]                                              # [Bq, k, L]
        return T[tq[:, None, :].expand_as(tr_sel), tr_sel].sum(-1)
    de, dt = exact(idx_e), exact(idx_t)
    kth = dt[:, -1:]
    out["cross_check"] = dict(
        queries=96, k=k,
        neighbours_within_exact_kth=round(float((de <= kth + 1.0).double().mean()), 6),
        same_exact_distance_multiset=bool(torch.allclose(de.sort(1).values, dt, rtol=0, atol=1.0)),
        index_overlap=round(float(sum(len(set(a) & set(b)) for a, b in zip(idx_e.tolist(), idx_t.tolist()))
                                  / idx_t.numel()), 4),
        max_rel_dist_err=round(float(((d_e.double() - de).abs() / de.clamp_min(1.0)).max()), 6),
        note="distance ties are broken by bf16 rounding in embedding space and by index in the token index, "
             "so index sets may differ at tied k-th distances; the exact-distance multisets must not")
    # reference-equivalent CPU: torch.cdist + topk (embedding_rag_dataset.py:390-402) on a sample
    threads = torch.get_num_threads()
    m = min(n, 512)
    Ec = eidx.rows(0, m).float().cpu()
    Qc = Q[:48].float().cpu()
    t0 = time.perf_counter()
    reps = 0
    while time.perf_counter() - t0 < 3.0:
        torch.topk(torch.cdist(Qc, Ec), min(k, m), dim=1, largest=False)
        reps += 1
    t_cpu = (time.perf_counter() - t0) / reps * (n / m)
    out["cpu_reference_equivalent"] = dict(
        queries=48, seconds_per_query_batch=round(t_cpu, 3), cores=threads, kind="reference-equivalent",
        sample=f"torch.cdist + topk of 48 f32 queries vs {m} panel rows x {L * D} dims, scaled x{n / m:.1f} to {n}")
    out["traffic"] = pmc_traffic("knn_emb_dot_kernel")
    out["gpu_vs_cpu_at_48"] = round(t_cpu / (out["per_queries"][0]["avg_launch_ms"] * 1e-3), 1)
    del eidx
    torch.cuda.empty_cache()
    return out


def pmc_traffic(kernel_name):
    """HBM bytes per launch (FETCH_SIZE x2 + WRITE_SIZE, rocprofv3 --pmc passes run by tools/pmc.sh
    on this bench, committed as profiles/pmc_traffic.json), launch-weighted over the kernel class."""
    f = REPO / "profiles" / "pmc_traffic.json"
    cls = {"rows_gemm_kernel": "gemm", "tailw_kernel": "ffn", "tail_kernel": "ffn", "ffn_kernel": "ffn", "attn32_bf16": "attention",
           "attn32_dma": "attention", "knn_emb_dot_kernel": "knn_emb"}
    key = next((v for k, v in cls.items() if kernel_name.startswith(k)), None)
    if key is None or not f.exists():
        return None
    ent = json.loads(f.read_text())["kernels"].get(key)
    if not ent:
        return None
    n = sum(e["launches"] for e in ent)
    fetch = sum(e["fetch_bytes"] * e["launches"] for e in ent) / n
    write = sum((e["write_bytes"] or 0) * e["launches"] for e in ent) / n
    return {"bytes_per_launch": round(fetch + write), "fetch_bytes": round(fetch), "write_bytes": round(write),
            "source": "profiles/pmc_traffic.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, FETCH x2 on gfx950)"}


def cpu_baseline(args, model, vocab, af_np, ref_af, raw_mask, x, dev):
    """Oracle ('port') timed on host cores: exact LUT-form kNN over a panel sample
    (scaled linearly to the full panel) + fp32 numpy forward of ONE sample."""
    from oracle import knn_np, model_np
    from src.dataset.synthetic import hash_uniform
    sd = {kk: v.detach().float().cpu().numpy() for kk, v in model.state_dict().items()}
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    S, k = args.window, args.k
    ns = min(args.cpu_panel, args.n_ref)
    r, c = np.meshgrid(np.arange(ns), np.arange(S), indexing="ij")
    panel = (hash_uniform(1234, r, c) < af_np[None]).astype(np.uint8)
    tok = np.concatenate([x["hap_1"][:1].cpu().numpy(), x["hap_2"][:1].cpu().numpy()])
    W = sd["bert.embedding.tokenizer.weight"]
    t0 = time.perf_counter()
    dq, _ = knn_np.quantize_lut(knn_np.lut_delta(W, tok, None, raw_mask.astype(np.uint8)), 2)
    idx, _ = knn_np.knn(panel, dq, k)
    t_knn = (time.perf_counter() - t0) * (args.n_ref / ns)
    ref_tok = vocab.tokenize(panel, np.zeros(1030, np.int64))
    xo = {kk: x[kk][:1].cpu().numpy() for kk in ("hap_1", "hap_2", "af", "af_p", "pos", "ref", "het", "hom")}
    xo["rag_mean_h1"] = model_np.rag_mean(ref_tok, idx[:1], ref_af, sd)
    xo["rag_mean_h2"] = model_np.rag_mean(ref_tok, idx[1:], ref_af, sd)
    t1 = time.perf_counter()
    model_np.forward(xo, sd, args.layers, args.heads)
    t_fwd = time.perf_counter() - t1
    masked = 2 * int(raw_mask.sum())
    return {"value": round(masked / (t_knn + t_fwd), 1), "unit": "masked SNVs/s", "cores": threads,
            "kind": "port",
            "sample": f"1 sample (2 haplotypes): oracle kNN over {ns} panel haplotypes scaled x{args.n_ref / ns:.1f} "
                      f"to {args.n_ref} ({t_knn:.2f}s) + numpy fp32 forward d{args.dims}/L{args.layers} ({t_fwd:.2f}s)"}


if __name__ == "__main__":
    main()
