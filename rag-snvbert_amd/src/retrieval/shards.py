"""Panel sharding across ranks.

Each rank holds a contiguous range of every window's panel haplotypes (``PanelShard``)
and serves the queries of ALL ranks against it; one retrieval step is

  1. all-gather the query tokens (u8, 1 B per position; plus the query AF rows when they
     differ from the panel's) — every rank then quantises the same LUTs;
  2. local exact top-k over the shard, keys carrying GLOBAL indices (``ref_offset``);
  3. all-gather the partial key lists and merge them with the same (distance, index)
     order: every key carries its global index and the order is total, so the merged
     top-k is identical to one GPU scanning the whole panel;
  4. the neighbour mean needs only the per-site alt-allele count over the k neighbours:
     each rank counts the neighbours it owns for all queries, an all-reduce (SUM, u8,
     nq_all x n_sites_pad bytes) completes the counts, each rank keeps its own rows.

In eval no neighbour codes or embeddings cross the links (a [nq, k, sites] code exchange
would be k times larger, a [nq, L, D] embedding reduction ~750x).  Train mode with dropout
needs each neighbour's own dropout mask and drop(e_q) in the distance, so there step 1 also
all-gathers the dropped-out query offsets and step 4 exchanges the codes of the unique
retrieved haplotypes instead of counts (sharded_neighbours ``aq_rows`` / ``want_codes``:
at C4, 48 queries x 1030 x 384 f32 = 76 MB per rank and <= 3 MB of codes).  The compute steps are
pluggable (``ShardOps``): the product uses the HIP kernels, the world-2 gloo test the
oracle's on the CPU, over the same collective plumbing.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Tuple

import torch
import torch.distributed as dist


@dataclass
class PanelShard:
    """This rank's contiguous haplotype range of an n-haplotype panel."""
    rank: int
    world: int
    group: Optional[object] = None

    def bounds(self, n: int) -> Tuple[int, int]:
        return n * self.rank // self.world, n * (self.rank + 1) // self.world

    @classmethod
    def current(cls, group=None) -> Optional["PanelShard"]:
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
            return None
        return cls(dist.get_rank(group), dist.get_world_size(group), group)


def _gloo(group) -> bool:
    return dist.get_backend(group) == "gloo"


def _all_gather(x: torch.Tensor, group=None) -> torch.Tensor:
    """[world, *x.shape]; gloo (CPU collectives, e.g. the world-2 tests — also with the ranks'
    tensors on one GPU) stages device tensors through the host."""
    world = dist.get_world_size(group)
    if _gloo(group):
        h = x.cpu()
        parts = [torch.empty_like(h) for _ in range(world)]
        dist.all_gather(parts, h, group=group)
        return torch.stack(parts).to(x.device)
    out = torch.empty((world,) + tuple(x.shape), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x, group=group)
    return out


def _all_reduce(x: torch.Tensor, op, group=None) -> torch.Tensor:
    if _gloo(group) and x.is_cuda:
        h = x.cpu()
        dist.all_reduce(h, op=op, group=group)
        x.copy_(h)
    else:
        dist.all_reduce(x, op=op, group=group)
    return x


def all_gather_rows(x: torch.Tensor, group=None) -> Tuple[torch.Tensor, List[int]]:
    """Concatenate every rank's ``x`` [n_r, ...] along dim 0 (n_r may differ): returns
    (x_all [sum n_r, ...], [n_0, ..., n_{w-1}])."""
    world = dist.get_world_size(group)
    sizes = [int(v) for v in _all_gather(torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device),
                                         group).view(-1).tolist()]
    nmax = max(sizes)
    if x.shape[0] < nmax:
        x = torch.cat([x, x.new_zeros((nmax - x.shape[0],) + tuple(x.shape[1:]))])
    out = _all_gather(x.contiguous(), group)
    return torch.cat([out[r, :sizes[r]] for r in range(world)]), sizes


def merge_keys_gathered(gathered: torch.Tensor, k: int,
                        merge_fn: Optional[Callable[[torch.Tensor, int], torch.Tensor]] = None) -> torch.Tensor:
    """gathered: [world, nq, k] key lists -> [nq, k].  merge_fn defaults to the HIP merge kernel."""
    if merge_fn is None:
        from .. import kernels as K
        merge_fn = K.topk_merge
    return merge_fn(gathered.contiguous(), k)


def sharded_search(local_keys: torch.Tensor, k: int, group=None,
                   merge_fn: Optional[Callable[[torch.Tensor, int], torch.Tensor]] = None) -> torch.Tensor:
    """All-gather every rank's [nq, k] local top-k keys (same queries on every rank) and merge."""
    world = dist.get_world_size(group)
    if world == 1:
        return local_keys
    # keys travel as their int64 bit pattern (no reduction is applied to them)
    out = _all_gather(local_keys.contiguous().view(torch.int64), group)
    return merge_keys_gathered(out.view(local_keys.dtype), k, merge_fn)


@dataclass
class ShardOps:
    """Compute steps of a sharded search (product: HIP kernels; tests: the oracle).

    keys(tok, af_rows) -> (keys [nq, k] uint64-as-int64 with global indices, exps, consts)
    merge(keys [n_lists, nq, k], k) -> [nq, k]
    decode(keys, exps, consts) -> (idx int64 [nq, k], dist f32 [nq, k])
    counts(idx [nq, k]) -> u8 [nq, ld]: alt-allele counts over the neighbours this shard owns
    codes(uniq [U]) -> u8 [U, ld]: the codes of the rows this shard owns, zero rows elsewhere
    (keys also takes a third argument, per-query embedding offsets [nq, L, D], when given)"""
    keys: Callable
    merge: Callable
    decode: Callable
    counts: Callable
    codes: Optional[Callable] = None


def batch_windows(windows, group=None) -> List[int]:
    """Union of the windows of every rank's batch, sorted: the order in which all ranks run
    their per-window collectives (a rank without queries of a window joins with none)."""
    world = dist.get_world_size(group)
    got: List[object] = [None] * world
    dist.all_gather_object(got, sorted(int(w) for w in windows), group=group)
    return sorted({w for g in got for w in g})


def any_rank(flag: bool, device, group=None) -> bool:
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device)
    return bool(_all_reduce(t, dist.ReduceOp.MAX, group).item())


def sharded_neighbours(tok: torch.Tensor, k: int, ops: ShardOps, af_rows: Optional[torch.Tensor] = None,
                       group=None, aq_rows: Optional[torch.Tensor] = None, want_codes: bool = False):
    """One sharded retrieval step for this rank's queries ``tok`` [nq, L] (token ids < 256).

    Returns (idx [nq, k] global panel indices, dist [nq, k], counts) for the rank's own
    queries.  ``counts`` is u8 [nq, ld] — the input of ``rag_mean(..., counts=)`` — or, with
    ``want_codes`` (train mode with dropout: every neighbour is re-encoded with its own
    dropout mask, embedding_rag_dataset.py:406-417), the pair (uniq, uniq_codes): the sorted
    global indices of every neighbour retrieved for ANY rank's query and their allele codes
    u8 [U, ld], assembled by one SUM all-reduce from the shards that own them (a code is 0/1
    and each row has exactly one owner).  ``aq_rows`` [nq, L, D] f32: per-query embedding
    offsets of the exact LUT form (train-mode queries embedded WITH dropout, :385-386) — they
    travel with the tokens so every shard ranks the same dropped-out query embeddings."""
    tok_all, sizes = all_gather_rows(tok.to(torch.uint8), group)
    af_all = all_gather_rows(af_rows.float(), group)[0] if af_rows is not None else None
    aq_all = all_gather_rows(aq_rows.float().contiguous(), group)[0] if aq_rows is not None else None
    keys, exps, consts = ops.keys(tok_all.long(), af_all, aq_all) if aq_all is not None else \
        ops.keys(tok_all.long(), af_all)
    merged = sharded_search(keys, k, group, ops.merge)
    idx, dst = ops.decode(merged, exps, consts)
    r = dist.get_rank(group)
    o = sum(sizes[:r])
    if want_codes:
        uniq = torch.unique(idx[idx >= 0])                   # identical on every rank
        codes = _all_reduce(ops.codes(uniq), dist.ReduceOp.SUM, group)
        extra = (uniq, codes)
    else:
        extra = _all_reduce(ops.counts(idx), dist.ReduceOp.SUM, group)[o:o + sizes[r]]
    return idx[o:o + sizes[r]], (dst[o:o + sizes[r]] if dst is not None else None), extra


def kernel_ops(index, W: torch.Tensor, site_mask: torch.Tensor, k: int, limbs: int = 2,
               aq_fn: Optional[Callable[[torch.Tensor], torch.Tensor]] = None,
               Ar: Optional[torch.Tensor] = None, Wp: Optional[torch.Tensor] = None) -> ShardOps:
    """The HIP kernels over this rank's ``PanelIndex`` shard.  With query AF rows, the LUTs
    take the exact A_q != A_r form (``aq_fn`` maps AF rows to their AF embeddings).  ``Wp``:
    the panel side's (cached) token table when it differs from ``W``."""
    from .. import kernels as K

    def keys(tok_all, af_all, aq_all=None):
        nq = tok_all.shape[0]
        if aq_all is not None:
            # per-query offsets (dropped-out train queries): Ar is the panel's AF embedding or 0
            ar = Ar if Ar is not None else torch.zeros(aq_all.shape[1:], device=aq_all.device)
            lut, exps, consts = index.lut(tok_all, W, site_mask, limbs, aq_all.contiguous(), nq, ar, Wp=Wp)
            return index.scan_keys(lut, nq, limbs, k), exps, consts
        if af_all is None:
            lut, exps, consts = index.lut(tok_all, W, site_mask, limbs, Wp=Wp)
            return index.scan_keys(lut, nq, limbs, k), exps, consts
        Aq = aq_fn(af_all)
        lut, exps, consts = index.lut(tok_all, W, site_mask, limbs, Aq, nq, Ar, Wp=Wp)
        return index.scan_keys(lut, nq, limbs, k), exps, consts

    def codes(uniq):
        i = uniq - index.ref_offset
        own = (i >= 0) & (i < index.codes.shape[0])
        out = torch.zeros(uniq.numel(), index.codes.shape[1], device=uniq.device, dtype=torch.uint8)
        out[own] = index.codes[i[own]]
        return out

    return ShardOps(keys=keys, merge=K.topk_merge, decode=K.knn_decode,
                    counts=lambda idx: K.neighbor_counts(idx, index.codes, index.ref_offset), codes=codes)
