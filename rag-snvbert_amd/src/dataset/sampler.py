"""Window-grouped samplers (reference: src/dataset/sampler.py:39-135 and
src/infer_embedding_rag.py:32-51).  Same index streams as the reference
(python ``random`` seeded identically), plus a rank-aware variant that keeps all
ranks on the same window in lock-step and splits that window's samples.
"""

from __future__ import annotations

import random
from typing import Iterator, Optional

from torch.utils.data import Sampler


class WindowGroupedSampler(Sampler):
    def __init__(self, dataset, shuffle: bool = True, seed: Optional[int] = None):
        self.dataset, self.shuffle, self.seed = dataset, shuffle, seed
        wc = dataset.window_count
        self.window_groups = {}
        for idx in range(len(dataset)):
            self.window_groups.setdefault(idx % wc, []).append(idx)
        self.num_samples = len(dataset)
        self.num_windows = len(self.window_groups)

    def __iter__(self) -> Iterator[int]:
        window_ids = list(self.window_groups.keys())
        if self.shuffle:
            if self.seed is not None:
                random.seed(self.seed)
            random.shuffle(window_ids)
        for w in window_ids:
            ids = self.window_groups[w].copy()
            if self.shuffle:
                random.shuffle(ids)
            yield from ids

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        if self.seed is not None:
            self.seed = self.seed + epoch      # reference behaviour (sampler.py:127-135)
            random.seed(self.seed)

    # the order of an epoch is a function of the (cumulative) seed alone: checkpointed with it
    def state_dict(self) -> dict:
        return {"seed": self.seed}

    def load_state_dict(self, state: dict) -> None:
        self.seed = state.get("seed", self.seed)


class WindowMajorSampler(Sampler):
    """infer_embedding_rag.py:32-51: yields s * num_windows + w, window-major."""

    def __init__(self, dataset):
        self.total_items = len(dataset)
        self.num_windows = dataset.window_count
        self.num_samples = self.total_items // self.num_windows

    def __iter__(self):
        for w in range(self.num_windows):
            for s in range(self.num_samples):
                yield s * self.num_windows + w

    def __len__(self):
        return self.total_items


class DistributedWindowSampler(Sampler):
    """Rank-aware WindowGroupedSampler (sampler.py:87-135 semantics across ranks).

    Every rank draws the same per-epoch permutation (private ``random.Random(seed + epoch)``,
    identical on all ranks): the window order is shuffled, then each window's samples; a
    window's list is padded by wrapping to a multiple of ``world`` (as torch's
    DistributedSampler pads) and rank r takes positions r, r + world, ...  So all ranks visit
    the windows in lock-step (one panel index per window live at a time), every rank yields
    exactly ``ceil(samples_per_window / world)`` items per window — equal batch counts, so
    the bucketed gradient all-reduce (and the sharded panel's per-window collectives) never
    wait on a rank that ran out — and the union over ranks covers every sample of every window.

    ``mark_padding`` (default: on for the unshuffled validation order): the wrapped duplicates
    are yielded as ``item + len(dataset)``, which the RAG datasets serve as the same sample with
    an all-zero metric mask (``EmbeddingRAGDataset.__getitem__``) — so no sample is counted twice
    in validation losses, F1 and early stopping, while every rank still runs the same number of
    batches."""

    def __init__(self, dataset, rank: int, world: int, shuffle: bool = True, seed: int = 42, window_order=None,
                 mark_padding: Optional[bool] = None):
        if not 0 <= rank < world:
            raise ValueError(f"rank {rank} outside world {world}")
        self.rank, self.world, self.shuffle, self.seed, self.epoch = rank, world, shuffle, seed, 0
        self.num_windows = dataset.window_count
        self.n_items = len(dataset)
        self.num_samples = self.n_items // self.num_windows
        if self.num_samples == 0:
            raise ValueError("dataset has fewer items than windows")
        self.order = list(window_order) if window_order is not None else None
        self.per_rank = (self.num_samples + world - 1) // world
        self.mark_padding = (not shuffle) if mark_padding is None else mark_padding

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def state_dict(self) -> dict:
        return {"epoch": self.epoch, "seed": self.seed}

    def load_state_dict(self, state: dict) -> None:
        self.epoch, self.seed = int(state.get("epoch", self.epoch)), int(state.get("seed", self.seed))

    def __iter__(self):
        rng = random.Random(self.seed + self.epoch)
        windows = list(self.order) if self.order is not None else list(range(self.num_windows))
        if self.shuffle and self.order is None:
            rng.shuffle(windows)
        total = self.per_rank * self.world
        for w in windows:
            samples = list(range(self.num_samples))
            if self.shuffle:
                rng.shuffle(samples)
            n = len(samples)
            samples = (samples * ((total + n - 1) // n))[:total]
            for pos in range(self.rank, total, self.world):
                item = samples[pos] * self.num_windows + w
                yield item + self.n_items if (self.mark_padding and pos >= n) else item

    def __len__(self):
        return self.per_rank * self.num_windows
