"""v18 embedding-RAG imputation entry point (reference: src/infer_embedding_rag.py:53-257).

Data: ``EmbeddingRAGInferDataset`` (InferDataset items over the panel's full site list;
the sites absent from the target are masked and imputed).  Per batch (window-major order,
WindowMajorSampler): retrieval on the HBM token index (exact int8-MFMA kNN, no FAISS, no
host round trip), the native eval forward, then the reference's post-processing on the
device (snvrag_infer_post: second softmax of the head probabilities, genotype products).
Results stay on the GPU until the end of the run; one device->host copy feeds the
geometry step ([W, S, L] -> [W*L, S], slice [1, 1+window), fit to the panel's site count —
infer_embedding_rag.py:166-203) and the writers.

Outputs (``--output_path``): ``imputed.npz`` (hap1/hap2 ALT probabilities, GP, mask,
positions) and ``imputed.vcf`` (the imputed sites = mask of the first sample, as
infer_embedding_rag.py:237; GT phased argmax, HDS, GP = (p00, p01 + p10, p11), DS,
``%.3f``).  The reference's VCF call fails with a TypeError, so the
writer here defines the output instead of mirroring it.

Windows: query windows are INFER_WINDOW_LEN = 1020 sites; ``--index_window_len`` 510
(default) reproduces the reference's 510-site index windows and infer masks
(embedding_rag_infer_dataset.py:16), 1020 aligns them with the query windows.
"""

from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch

INFER_WINDOW_LEN = 1020
MAX_SEQ_LEN = 1030


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="v18 embedding-RAG imputation (MI355X)")
    for name in ("ref_panel", "infer_dataset", "infer_panel", "freq_path", "type_path", "pop_path", "pos_path"):
        p.add_argument(f"--{name}", type=str, default=None)
    p.add_argument("-c", "--check_point", type=str, default=None,
                   help="the reference's pickled model or a state_dict (read without executing pickled code)")
    p.add_argument("-o", "--output_path", type=str, default="output/infer")
    p.add_argument("--chrom", type=str, default="21")
    p.add_argument("-d", "--dims", type=int, default=384)
    p.add_argument("-l", "--layers", type=int, default=12)
    p.add_argument("-a", "--attn_heads", type=int, default=12)
    p.add_argument("-b", "--infer_batch_size", type=int, default=32)
    p.add_argument("-n", "--num_workers", type=int, default=0)
    p.add_argument("--k_retrieve", type=int, default=1)
    p.add_argument("--cuda_devices", type=int, nargs="+", default=None)
    p.add_argument("--window_len", type=int, default=INFER_WINDOW_LEN)
    p.add_argument("--index_window_len", type=int, default=510,
                   help="510: the reference's index windows (compat); 1020: aligned with the query windows")
    p.add_argument("--dtype", choices=["bf16", "f32"], default="bf16")
    p.add_argument("--synthetic", type=int, default=0, help="samples of in-memory synthetic data")
    p.add_argument("--synthetic_sites", type=int, default=2040, help="synthetic: panel sites")
    p.add_argument("--synthetic_ref", type=int, default=256, help="synthetic: panel samples")
    p.add_argument("--mask_rate", type=float, default=0.3,
                   help="synthetic: fraction of panel sites absent from the target (C5 sweep 0.1..0.9)")
    p.add_argument("--no_vcf", action="store_true")
    p.add_argument("--seed", type=int, default=0, help="weight init without --check_point (synthetic runs)")
    p.add_argument("--dist_backend", default="nccl", choices=["nccl", "gloo"],
                   help="WORLD_SIZE > 1 (torch.distributed.run, one process per GPU): nccl (= RCCL) or gloo "
                        "(host-staged: the multi-rank tests with every rank on one GPU)")
    return p.parse_args(argv)


def postprocess(probs_h1: torch.Tensor, probs_h2: torch.Tensor):
    """Device post-processing of one batch -> (p1 [B, L], p2 [B, L], gt [B, L, 4])."""
    from . import kernels as K
    return K.infer_post(probs_h1, probs_h2)


def geometry(h1, h2, gt, mask, n_windows: int, n_variants: int, window_len: int):
    """infer_embedding_rag.py:171-203 on stacked [W*S, L] arrays (window-major order)."""
    h1, h2 = h1[:, 1:1 + window_len], h2[:, 1:1 + window_len]
    gt, mask = gt[:, 1:1 + window_len], mask[:, 1:1 + window_len]
    S = h1.shape[0] // n_windows
    Lw = h1.shape[1]
    tr = lambda a: a.reshape(n_windows, S, Lw, *a.shape[2:]).swapaxes(1, 2).reshape(n_windows * Lw, S, *a.shape[2:])
    h1, h2, gt, mask = tr(h1), tr(h2), tr(gt), tr(mask)
    if h1.shape[0] >= n_variants:
        return h1[:n_variants], h2[:n_variants], gt[:n_variants], mask[:n_variants]
    pad = n_variants - h1.shape[0]
    padf = lambda a: np.pad(a, ((0, pad),) + ((0, 0),) * (a.ndim - 1))
    return padf(h1), padf(h2), padf(gt), padf(mask)


GT_MAP = ("0|0", "0|1", "1|0", "1|1")       # src/dataset/utils.py:15-20


def vcf_cells(h1, h2, gt):
    """Per-sample FORMAT cells GT:HDS:GP:DS of one site, as generate_vcf_efficient_optimized
    writes them (src/dataset/utils.py:406-461): GT = GT_MAP[argmax gt], HDS = (p1, p2),
    GP = (p00, p01 + p10, p11), DS = GP1 + 2 GP2, all '%.3f'."""
    g = np.argmax(gt, -1)
    gp0, gp1, gp2 = gt[..., 0], gt[..., 1] + gt[..., 2], gt[..., 3]
    ds = gp1 + 2 * gp2
    return [f"{GT_MAP[g[s]]}:{h1[s]:.3f},{h2[s]:.3f}:{gp0[s]:.3f},{gp1[s]:.3f},{gp2[s]:.3f}:{ds[s]:.3f}"
            for s in range(len(h1))]


def write_vcf(path, chrom, pos, h1, h2, gt, samples, pos_flag=None, ref=None, alt=None):
    """VCF 4.2 records of the imputed sites (utils.py:378-479 layout: FORMAT GT:HDS:GP:DS,
    ID '.', REF/ALT '.' unless given, QUAL 0, FILTER PASS).  ``pos_flag`` selects the sites
    written (the reference writes only flagged = imputed positions, infer_embedding_rag.py:237)."""
    with open(path, "w") as f:
        f.write("##fileformat=VCFv4.2\n##source=rag-snvbert_amd\n")
        f.write('##FORMAT=<ID=GT,Number=1,Type=String,Description="Genotype (argmax of GP)">\n')
        f.write('##FORMAT=<ID=HDS,Number=2,Type=Float,Description="Haplotype ALT dosages">\n')
        f.write('##FORMAT=<ID=GP,Number=3,Type=Float,Description="Genotype probabilities">\n')
        f.write('##FORMAT=<ID=DS,Number=1,Type=Float,Description="ALT dosage">\n')
        f.write("#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" + "\t".join(samples) + "\n")
        for i in range(len(pos)):
            if pos_flag is not None and not pos_flag[i]:
                continue
            r = ref[i] if ref is not None else "."
            a = alt[i] if alt is not None else "."
            f.write(f"{chrom}\t{int(pos[i])}\t.\t{r}\t{a}\t0.0\tPASS\t.\tGT:HDS:GP:DS\t" +
                    "\t".join(vcf_cells(h1[i], h2[i], gt[i])) + "\n")


def build_dataset(args):
    from .dataset.embedding_rag_infer_dataset import EmbeddingRAGInferDataset
    from .dataset.vocab import WordVocab
    if not args.synthetic:
        from .dataset.dataset import PanelData
        vocab = WordVocab(list(PanelData.from_file(args.infer_panel).pop_class_dict.keys()))
        ds = EmbeddingRAGInferDataset.from_file(vocab, args.infer_dataset, args.infer_panel, args.freq_path,
                                                args.type_path, args.pop_path, args.pos_path,
                                                ref_vcf_path=args.ref_panel, window_len=args.window_len,
                                                index_window_len=args.index_window_len)
        return ds, vocab
    from .dataset.synthetic import make_infer_arrays, make_infer_dataset
    a = make_infer_arrays(args.synthetic_sites, args.synthetic, args.synthetic_ref, missing_rate=args.mask_rate,
                          seed=11)
    return make_infer_dataset(a, index_window_len=args.index_window_len)


def rank_rows(n_rows: int, rank: int, world: int):
    """The contiguous slice of the window-major sampler stream rank ``rank`` imputes: whole
    sample-windows, ranks in stream order, so each rank touches few windows (few panel-index
    builds) and the gather is a concatenation in rank order."""
    return n_rows * rank // world, n_rows * (rank + 1) // world


def _gather_rows(t: torch.Tensor, sizes, group=None) -> torch.Tensor:
    """Concatenate every rank's rows (ragged counts ``sizes``) in rank order."""
    from .retrieval.shards import _all_gather
    pad = max(sizes)
    if t.shape[0] < pad:
        t = torch.cat([t, t.new_zeros((pad - t.shape[0],) + tuple(t.shape[1:]))])
    g = _all_gather(t.contiguous(), group)
    return torch.cat([g[r, :n] for r, n in enumerate(sizes)])


def run(ds, model, dev, batch_size: int, k: int, num_workers: int = 0, window_len: int = INFER_WINDOW_LEN,
        group=None):
    """The inference loop (infer_embedding_rag.py:132-157) and geometry (:165-203) over ``ds``
    with an eval ``model`` on ``dev``.  Returns host arrays h1/h2 [n_sites, S], gt
    [n_sites, S, 4], mask [n_sites, S], the neighbour indices per sampler row and the time.

    Several ranks (``torch.distributed`` initialised, configs[4]): the panel is replicated,
    rank r imputes rows ``rank_rows`` of the window-major stream (batches formed inside its
    slice), and the per-row outputs are all-gathered in stream order before the geometry — the
    same arrays as one process (every row's retrieval and forward depend on that row alone).
    ``seconds`` is the slowest rank's loop time."""
    from .dataset.embedding_rag_dataset import embedding_rag_collate_fn
    from .dataset.sampler import WindowMajorSampler
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if world > 1 else 0
    emb = model.bert.embedding
    order = list(iter(WindowMajorSampler(ds)))
    lo, hi = rank_rows(len(order), rank, world)
    loader = torch.utils.data.DataLoader(ds, batch_size=batch_size, sampler=order[lo:hi],
                                         num_workers=num_workers, collate_fn=embedding_rag_collate_fn)
    outs = {"h1": [], "h2": [], "gt": [], "mask": [], "idx1": [], "idx2": []}
    t0 = time.perf_counter()
    with torch.no_grad():
        for batch in loader:
            batch = ds.process_batch_retrieval(batch, emb, dev, k)
            x = {key: (v.to(dev, non_blocking=True) if torch.is_tensor(v) else v) for key, v in batch.items()}
            out = model(x)
            p1, p2, gt = postprocess(out[0], out[1])
            outs["h1"].append(p1)
            outs["h2"].append(p2)
            outs["gt"].append(gt)
            outs["mask"].append(x["mask"])
            outs["idx1"].append(x["rag_idx_h1"])
            outs["idx2"].append(x["rag_idx_h2"])
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        sizes = [rank_rows(len(order), r, world)[1] - rank_rows(len(order), r, world)[0] for r in range(world)]
        full = {}
        for key, v in outs.items():
            loc = torch.cat(v) if v else _empty_rows(key, dev, k)
            loc = loc.long() if key in ("idx1", "idx2", "mask") else loc.float()   # one dtype on every rank
            full[key] = _gather_rows(loc, sizes, group)
        outs = {key: [t] for key, t in full.items()}
        from .retrieval.shards import _all_reduce
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        elapsed = float(_all_reduce(t, dist.ReduceOp.MAX, group).item())
    host = {key: torch.cat(v).cpu().numpy() for key, v in outs.items()}
    h1, h2, gt, mask = geometry(host["h1"], host["h2"], host["gt"], host["mask"], ds.window_count,
                                len(ds.ori_pos), window_len)
    return dict(h1=h1, h2=h2, gt=gt, mask=mask, idx1=host["idx1"], idx2=host["idx2"], seconds=elapsed,
                masked_snvs=int(host["mask"].sum()) * 2, batch_mask=host["mask"], batch_h1=host["h1"],
                batch_h2=host["h2"])


def _empty_rows(key, dev, k):
    """A rank with no rows (more ranks than sample-windows) contributes zero-row tensors."""
    shape = {"gt": (0, MAX_SEQ_LEN, 4), "idx1": (0, k), "idx2": (0, k)}.get(key, (0, MAX_SEQ_LEN))
    dt = torch.long if key in ("idx1", "idx2", "mask") else torch.float32
    return torch.zeros(shape, device=dev, dtype=dt)


def infer(argv=None):
    args = parse_args(argv)
    if not torch.cuda.is_available():
        raise SystemExit("imputation runs on the MI355X kernels only (no CPU fallback)")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dev = torch.device(f"cuda:{int(os.environ.get('LOCAL_RANK', '0'))}")
    else:
        dev = torch.device(f"cuda:{args.cuda_devices[0] if args.cuda_devices else torch.cuda.current_device()}")
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    from .engine import engine_for
    from .model import build_model
    ds, vocab = build_dataset(args)
    torch.manual_seed(args.seed)          # every rank (and every run) builds the same random-init weights
    model = build_model(len(vocab), args.dims, args.layers, args.attn_heads)
    if args.check_point:
        # a trainer checkpoint of either build: the reference's pickled module (its classes
        # stubbed, nothing executed), a state_dict / {'state_dict'} / {'model'} (model/checkpoint.py)
        from .model.checkpoint import load_state_dict_any
        sd = load_state_dict_any(args.check_point)
        # strict: a missing or renamed key must not silently impute with random-init weights
        # (the reference loads with strict=False, infer_embedding_rag.py:99)
        model.load_state_dict(sd, strict=True)
    model = model.to(dev).eval()
    engine_for(model).set_dtype(torch.bfloat16 if args.dtype == "bf16" else torch.float32)
    res = run(ds, model, dev, args.infer_batch_size, args.k_retrieve, args.num_workers, args.window_len)
    h1, h2, gt, mask = res["h1"], res["h2"], res["gt"], res["mask"]
    if rank != 0:                      # the gathered arrays are written once
        return res
    os.makedirs(args.output_path, exist_ok=True)
    np.savez_compressed(os.path.join(args.output_path, "imputed.npz"), hap1=h1, hap2=h2, gp=gt, mask=mask,
                        pos=np.asarray(ds.ori_pos))
    if not args.no_vcf:
        samples = [f"S{i}" for i in range(h1.shape[1])]
        write_vcf(os.path.join(args.output_path, "imputed.vcf"), args.chrom, ds.ori_pos, h1, h2, gt, samples,
                  pos_flag=mask[:, 0].astype(bool))
    print(f"imputed {len(ds)} sample-windows in {res['seconds']:.2f}s "
          f"({res['masked_snvs'] / res['seconds']:.0f} masked SNVs/s)", flush=True)
    return res


if __name__ == "__main__":
    infer(sys.argv[1:])
