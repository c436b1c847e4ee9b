"""v18 embedding-RAG imputation entry point (reference: src/infer_embedding_rag.py:53-257).

Per batch (window-major order, WindowMajorSampler): retrieval on the HBM token index
(exact int8-MFMA kNN, no FAISS, no host round trip), the native eval forward, then the
reference's post-processing on the device (snvrag_infer_post: second softmax of the head
probabilities, genotype products).  Results stay on the GPU until the end of the run;
one device->host copy feeds the geometry step ([W, S, L] -> [W*L, S], slice [1, 1+window),
fit to the variant count — infer_embedding_rag.py:166-203) and the writers.

Outputs (``--output_path``): ``imputed.npz`` (hap1/hap2 ALT probabilities, GP, mask,
positions) and ``imputed.vcf`` (GT phased at p > 0.5, DS = p1 + p2, GP = (p00, p01 + p10,
p11), ``%.3f``).  The reference's VCF call fails with a TypeError, so the
writer here defines the output instead of mirroring it.

Windows: the reference's query windows are INFER_WINDOW_LEN = 1020 sites while its FAISS
index windows are 510 (embedding_rag_infer_dataset.py:16), misaligning index and query for
w > 0.  Here index and query share the dataset's windows (aligned); ``--window_len``
sets the slice length (1020, the reference's query geometry).
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
    p.add_argument("-c", "--check_point", type=str, default=None, help="state_dict checkpoint (weights_only load)")
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
    p.add_argument("--dtype", choices=["bf16", "f32"], default="bf16")
    p.add_argument("--synthetic", type=int, default=0, help="samples of in-memory synthetic data")
    p.add_argument("--synthetic_windows", type=int, default=2)
    p.add_argument("--synthetic_ref", type=int, default=256)
    p.add_argument("--mask_rate", type=float, default=None, help="synthetic: fixed mask level 0.1..0.9 (C5 sweep)")
    p.add_argument("--no_vcf", action="store_true")
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
    if not args.synthetic:
        raise SystemExit("reading the reference's VCF/H5 inputs needs scikit-allel/h5py, absent in this image; "
                         "run with --synthetic N (in-memory data with the same file contract)")
    from .dataset.synthetic import make_rag_dataset
    ds, vocab = make_rag_dataset(args.synthetic, args.window_len, args.synthetic_windows, args.synthetic_ref,
                                 seed=11, name="infer")
    if args.mask_rate is not None:
        from .dataset.utils import sequence_padding
        for w in range(ds.window_count):
            n = ds.window_actual_lens[w]
            rng = np.random.default_rng(1000 + w)
            raw = (rng.random(n) < args.mask_rate).astype(np.int64)
            ds.raw_window_masks[w] = raw
            ds.window_masks[w] = sequence_padding(raw, "int")
        ds.fixed_masks = True
    return ds, vocab


def infer(argv=None):
    args = parse_args(argv)
    if not torch.cuda.is_available():
        raise SystemExit("imputation runs on the MI355X kernels only (no CPU fallback)")
    dev = torch.device(f"cuda:{args.cuda_devices[0] if args.cuda_devices else torch.cuda.current_device()}")
    torch.cuda.set_device(dev)
    from .dataset.embedding_rag_dataset import embedding_rag_collate_fn
    from .dataset.sampler import WindowMajorSampler
    from .engine import engine_for
    from .model import build_model
    ds, vocab = build_dataset(args)
    model = build_model(len(vocab), args.dims, args.layers, args.attn_heads)
    if args.check_point:
        ck = torch.load(args.check_point, map_location="cpu", weights_only=True)
        sd = ck.get("model", ck) if isinstance(ck, dict) else ck
        sd = {k.replace("module.", ""): v for k, v in sd.items()}
        # strict: a missing or renamed key must not silently impute with random-init weights
        # (the reference loads with strict=False, infer_embedding_rag.py:99)
        model.load_state_dict(sd, strict=True)
    model = model.to(dev).eval()
    engine_for(model).set_dtype(torch.bfloat16 if args.dtype == "bf16" else torch.float32)
    emb = model.bert.embedding
    loader = torch.utils.data.DataLoader(ds, batch_size=args.infer_batch_size, sampler=WindowMajorSampler(ds),
                                         num_workers=args.num_workers, collate_fn=embedding_rag_collate_fn)
    outs = {"h1": [], "h2": [], "gt": [], "mask": []}
    t0 = time.perf_counter()
    with torch.no_grad():
        for batch in loader:
            if getattr(ds, "fixed_masks", False):     # C5 sweep: the window mask is the query mask
                w = int(batch["window_idx"][0])
                m = torch.from_numpy(np.asarray(ds.window_masks[w])).long()
                batch["mask"] = m.expand_as(batch["hap_1"]).clone()
                keep = batch["mask"] == 0
                batch["hap_1"] = torch.where(keep, batch["hap_1"], torch.full_like(batch["hap_1"], 4))
                batch["hap_2"] = torch.where(keep, batch["hap_2"], torch.full_like(batch["hap_2"], 4))
            batch = ds.process_batch_retrieval(batch, emb, dev, args.k_retrieve)
            x = {k: (v.to(dev, non_blocking=True) if torch.is_tensor(v) else v) for k, v in batch.items()}
            out = model(x)
            p1, p2, gt = postprocess(out[0], out[1])
            outs["h1"].append(p1)
            outs["h2"].append(p2)
            outs["gt"].append(gt)
            outs["mask"].append(x["mask"])
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    host = {k: torch.cat(v).cpu().numpy() for k, v in outs.items()}
    n_windows = ds.window_count
    n_variants = len(ds.pos)
    h1, h2, gt, mask = geometry(host["h1"], host["h2"], host["gt"], host["mask"], n_windows, n_variants,
                                args.window_len)
    os.makedirs(args.output_path, exist_ok=True)
    np.savez_compressed(os.path.join(args.output_path, "imputed.npz"), hap1=h1, hap2=h2, gp=gt, mask=mask,
                        pos=np.asarray(ds.pos))
    if not args.no_vcf:
        samples = [f"S{i}" for i in range(h1.shape[1])]
        write_vcf(os.path.join(args.output_path, "imputed.vcf"), args.chrom, ds.pos, h1, h2, gt, samples)
    masked = int(host["mask"].sum()) * 2
    print(f"imputed {len(ds)} sample-windows in {elapsed:.2f}s ({masked / elapsed:.0f} masked SNVs/s)", flush=True)
    return dict(h1=h1, h2=h2, gt=gt, mask=mask, seconds=elapsed, masked_snvs=masked)


if __name__ == "__main__":
    infer(sys.argv[1:])
