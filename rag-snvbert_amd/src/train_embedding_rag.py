"""v18 embedding-RAG training entry point (reference: src/train_embedding_rag.py:23-420).

Same command-line surface as the reference (dataset/panel/freq/window/type/pop/pos paths,
model and optimiser hyper-parameters, rag_k, resume, output) plus:
  --synthetic N_SAMPLES   build the data in memory (src/dataset/synthetic.py) — this image
                          has no 1000-Genomes files and no h5py/allel to read them;
  --max_steps N           stop an epoch after N batches (smoke runs).
Multi-GPU: launch one process per GPU with torch.distributed.run; ranks walk the windows
in lock-step (DistributedWindowSampler), sum gradients with bucketed RCCL all-reduces
(src/main/optimizer.py: the reference's DataParallel gradient over the global batch), sum
the epoch metrics over ranks and stop early together (main/pretrain_with_val_optimized.py).
"""

from __future__ import annotations

import argparse
import os
import sys

import torch


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="v18 embedding-RAG SNV imputation training (MI355X)")
    for name in ("train_dataset", "train_panel", "val_dataset", "val_panel", "refpanel_path", "freq_path",
                 "window_path", "type_path", "pop_path", "pos_path"):
        p.add_argument(f"--{name}", type=str, default=None)
    p.add_argument("--dims", type=int, default=384)
    p.add_argument("--layers", type=int, default=12)
    p.add_argument("--attn_heads", type=int, default=12)
    p.add_argument("--epochs", type=int, default=20)
    p.add_argument("--train_batch_size", type=int, default=24)
    p.add_argument("--val_batch_size", type=int, default=48)
    p.add_argument("--lr", type=float, default=7.5e-5)
    p.add_argument("--warmup_steps", type=int, default=15000)
    p.add_argument("--grad_accum_steps", type=int, default=2)
    p.add_argument("--focal_gamma", type=float, default=2.0)
    p.add_argument("--use_recon_loss", type=str, default="false")
    p.add_argument("--patience", type=int, default=5)
    p.add_argument("--val_metric", type=str, default="f1")
    p.add_argument("--min_delta", type=float, default=0.001)
    p.add_argument("--rag_k", type=int, default=1)
    p.add_argument("--cuda_devices", type=int, default=0)
    p.add_argument("--num_workers", type=int, default=0)
    p.add_argument("--resume_path", type=str, default=None)
    p.add_argument("--resume_epoch", type=int, default=None,
                   help="epoch to resume at (reference: default 0); unset = after a checkpoint of this "
                        "trainer's own epoch, 0 for a reference-format file")
    p.add_argument("--output_path", type=str, default="output/rag_bert.model")
    p.add_argument("--log_freq", type=int, default=500)
    p.add_argument("--rare_threshold", type=float, default=0.05)
    p.add_argument("--metrics_csv", type=str, default=None)
    p.add_argument("--weight_decay", type=float, default=0.01)
    p.add_argument("--synthetic", type=int, default=0, help="samples of in-memory synthetic data (0 = files)")
    p.add_argument("--synthetic_sites", type=int, default=1020)
    p.add_argument("--synthetic_windows", type=int, default=2)
    p.add_argument("--synthetic_ref", type=int, default=256, help="panel samples (2 haplotypes each)")
    p.add_argument("--max_steps", type=int, default=0)
    p.add_argument("--panel", default="sharded", choices=["sharded", "replicated"],
                   help="DDP: each rank holds 1/world of every window's panel and serves every rank's "
                        "queries (SURVEY §8e), or every rank holds the whole panel")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--dropout", type=float, default=0.1,
                   help="model dropout (the reference's BERT default 0.1); another value sets every dropout layer")
    p.add_argument("--dist_backend", default="nccl", choices=["nccl", "gloo"],
                   help="process-group backend for WORLD_SIZE > 1: nccl (= RCCL, one GPU per rank) or "
                        "gloo (host-staged collectives: the multi-rank tests with all ranks on one GPU)")
    return p.parse_args(argv)


def build_data(args, rank: int, world: int):
    from .dataset.embedding_rag_dataset import embedding_rag_collate_fn
    from .dataset.sampler import DistributedWindowSampler, WindowGroupedSampler
    if args.synthetic:
        from .dataset.synthetic import make_rag_dataset
        train, vocab = make_rag_dataset(args.synthetic, args.synthetic_sites, args.synthetic_windows,
                                        args.synthetic_ref, seed=args.seed, name="train")
        val, _ = make_rag_dataset(max(2, args.synthetic // 4), args.synthetic_sites, args.synthetic_windows,
                                  args.synthetic_ref, seed=args.seed + 1, name="val")
    else:
        raise SystemExit("reading the reference's H5/VCF inputs needs h5py and scikit-allel, which this image "
                         "does not have; run with --synthetic N (in-memory data with the same file contract)")
    mk = lambda ds, sampler, bs: torch.utils.data.DataLoader(ds, batch_size=bs, sampler=sampler,
                                                             num_workers=args.num_workers,
                                                             collate_fn=embedding_rag_collate_fn)
    # train_embedding_rag.py:218, :260 — seed 42 for the train order, deterministic validation
    if world > 1:
        ts = DistributedWindowSampler(train, rank, world, shuffle=True, seed=42)
        vs = DistributedWindowSampler(val, rank, world, shuffle=False)
        if args.panel == "sharded":
            from .retrieval.shards import PanelShard
            for ds in (train, val):
                ds.set_panel_shard(PanelShard.current())
    else:
        ts, vs = WindowGroupedSampler(train, shuffle=True, seed=42), WindowGroupedSampler(val, shuffle=False)
    return mk(train, ts, args.train_batch_size), mk(val, vs, args.val_batch_size), vocab


def main(argv=None):
    args = parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(args.cuda_devices)))
    if not torch.cuda.is_available():
        raise SystemExit("training runs on the MI355X kernels only (no CPU fallback)")
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    torch.manual_seed(args.seed + rank)
    # the datasets' construction-time window masks draw from numpy's global RNG (unseeded in the
    # reference, embedding_rag_dataset.py:160-170): seeded here so a run is reproducible (ranks
    # take rank 0's masks anyway, set_panel_shard)
    import numpy as np
    np.random.seed(args.seed)
    train_loader, val_loader, vocab = build_data(args, rank, world)
    from .main.pretrain_with_val_optimized import BERTTrainerWithValidationOptimized
    from .model import build_model
    model = build_model(len(vocab), args.dims, args.layers, args.attn_heads, dropout=args.dropout).to(dev)
    if args.dropout != 0.1:
        # every dropout layer, including the ones the reference fixes at 0.1 (fusion.py af_adapter /
        # fusion, foundation_model.py GenotypeClassifier FeedForward)
        for mod in model.modules():
            if isinstance(mod, torch.nn.Dropout):
                mod.p = args.dropout
    if world > 1:   # identical initial weights on every rank
        import torch.distributed as dist
        for t in list(model.parameters()) + list(model.buffers()):
            if args.dist_backend == "gloo":
                h = t.data.cpu()
                dist.broadcast(h, 0)
                t.data.copy_(h)
            else:
                dist.broadcast(t.data, 0)
    trainer = BERTTrainerWithValidationOptimized(
        model, train_loader, val_loader, vocab, lr=args.lr, weight_decay=args.weight_decay,
        warmup_steps=args.warmup_steps, log_freq=args.log_freq, grad_accum_steps=args.grad_accum_steps,
        focal_gamma=args.focal_gamma, use_recon_loss=args.use_recon_loss.lower() == "true",
        patience=args.patience, val_metric=args.val_metric, min_delta=args.min_delta,
        rare_threshold=args.rare_threshold, output_csv=args.metrics_csv if rank == 0 else None)
    trainer.rag_k = args.rag_k
    start = 0
    if args.resume_path:
        # train_embedding_rag.py:155-191 (weights; here also optimizer / schedule / early-stopping /
        # sampler state).  An explicit --resume_epoch (0 included) wins, as in the reference; unset,
        # a checkpoint of this trainer resumes after its epoch and a reference-format file (pickled
        # module, state_dict, {'state_dict': ...}: no trustworthy epoch) at the reference's default 0
        ep = trainer.load(args.resume_path)
        start = args.resume_epoch if args.resume_epoch is not None else \
            (ep + 1 if trainer.loaded_own_checkpoint else 0)
    ds, val_ds = train_loader.dataset, val_loader.dataset
    if start > 0 and hasattr(ds, "add_level"):
        # :326-336 — the curriculum level of the resumed epoch, min(start // 2, 7)
        for _ in range(min(start // 2, 7)):
            ds.add_level()
    if args.max_steps:
        import itertools

        class _Cap:
            def __init__(self, dl, n):
                self.dl, self.n, self.dataset, self.sampler = dl, n, dl.dataset, dl.sampler

            def __iter__(self):
                return itertools.islice(iter(self.dl), self.n)

        trainer.train_data = _Cap(train_loader, args.max_steps)
        trainer.val_data = _Cap(val_loader, args.max_steps)
    for epoch in range(start, args.epochs):                    # train_embedding_rag.py:343-434
        if hasattr(train_loader.sampler, "set_epoch"):      # :349-351
            train_loader.sampler.set_epoch(epoch)
        for d in (ds, val_ds):                                 # :354-357
            d.current_epoch = epoch
        if epoch > 0:
            # :360-389 — fresh training masks (the validation masks stay fixed), JIT caches reset
            if hasattr(ds, "regenerate_masks"):
                ds.regenerate_masks(seed=epoch)
            ds.jit_cache_win_idx = -1
            val_ds.jit_cache_win_idx = -1
        trainer.train(epoch)
        res = trainer.validate(epoch)
        if hasattr(val_ds, "clear_jit_cache"):                # :398-402
            val_ds.clear_jit_cache()
        # :405-406 — "best" is decided BEFORE this epoch's early-stopping update, i.e. from the
        # previous validation (the reference's order, kept for identical .best.pth semantics)
        trainer.save(epoch, args.output_path, is_best=trainer.epochs_no_improve == 0)
        if trainer.should_stop_early(res, epoch):
            break
        if (epoch + 1) % 2 == 0 and hasattr(ds, "add_level"):  # :418-430, capped at the last level
            ds.add_level()
    return trainer


if __name__ == "__main__":
    main(sys.argv[1:])
