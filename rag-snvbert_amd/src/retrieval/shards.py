"""Panel sharding across ranks: each rank holds a contiguous
range of panel haplotypes, computes its exact local top-k with GLOBAL indices
(ref_offset), the partial lists are all-gathered over RCCL (xGMI) and merged
with the same (distance, index) order — identical to the single-GPU result
because every key carries its global index.
"""

from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist


def merge_keys_gathered(gathered: torch.Tensor, k: int,
                        merge_fn: Optional[Callable[[torch.Tensor, int], torch.Tensor]] = None) -> torch.Tensor:
    """gathered: [world, nq, k] key lists -> [nq, k].  merge_fn defaults to the HIP merge kernel."""
    if merge_fn is None:
        from .. import kernels as K
        merge_fn = K.topk_merge
    return merge_fn(gathered.contiguous(), k)


def sharded_search(local_keys: torch.Tensor, k: int, group=None,
                   merge_fn: Optional[Callable[[torch.Tensor, int], torch.Tensor]] = None) -> torch.Tensor:
    """All-gather every rank's [nq, k] local top-k keys and merge them (one collective per batch)."""
    world = dist.get_world_size(group)
    if world == 1:
        return local_keys
    # keys travel as their int64 bit pattern (collectives have no uint64 reduction need here)
    src = local_keys.contiguous().view(torch.int64)
    out = torch.empty((world,) + tuple(src.shape), dtype=torch.int64, device=src.device)
    if dist.get_backend(group) == "gloo":
        dist.all_gather(list(out.unbind(0)), src, group=group)
    else:
        dist.all_gather_into_tensor(out, src, group=group)
    return merge_keys_gathered(out.view(local_keys.dtype), k, merge_fn)
