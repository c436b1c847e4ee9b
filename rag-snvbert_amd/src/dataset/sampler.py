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
    """Rank-aware window-major order: every rank visits windows in the same order and
    takes a contiguous share of each window's samples, so the per-window panel index
    (and its kNN shard) is the same on all ranks at the same time."""

    def __init__(self, dataset, rank: int, world: int, window_order=None):
        self.rank, self.world = rank, world
        self.num_windows = dataset.window_count
        self.num_samples = len(dataset) // self.num_windows
        self.order = list(window_order) if window_order is not None else list(range(self.num_windows))

    def _share(self):
        per = (self.num_samples + self.world - 1) // self.world
        lo = min(self.num_samples, self.rank * per)
        return range(lo, min(self.num_samples, lo + per))

    def __iter__(self):
        share = self._share()
        for w in self.order:
            for s in share:
                yield s * self.num_windows + w

    def __len__(self):
        return len(self._share()) * self.num_windows
