"""Featurisation helpers restated from ``src/dataset/utils.py`` and the AF-guided
mask of ``src/dataset/embedding_rag_dataset.py``.
"""

from __future__ import annotations

import numpy as np

MAX_SEQ_LEN = 1030
INFER_WINDOW_LEN = 1020
RARE_AF_THRESHOLD = 0.05     # embedding_rag_dataset.py:157
RARE_MASK_RATE = 0.7         # embedding_rag_dataset.py:158
MASK_RATES = (0.30, 0.40, 0.50, 0.60, 0.70, 0.80)   # dataset.py:252


def sequence_padding(seq: np.ndarray, dtype: str = "int", seq_len: int = MAX_SEQ_LEN) -> np.ndarray:
    """``VCFProcessingModule.sequence_padding`` (utils.py:121-132): one leading
    pad slot (aligned with <sos>), the data, then pads up to ``seq_len``."""
    seq = np.asarray(seq)
    pad = 0 if dtype == "int" else 0.0
    out_dtype = np.int64 if dtype == "int" else np.float64
    out = np.full(seq.shape[:-1] + (seq_len,), pad, dtype=out_dtype)
    out[..., 1:1 + seq.shape[-1]] = seq
    return out


def position_normalize(pos: np.ndarray) -> np.ndarray:
    """``VCFProcessingModule.position_normalize`` (utils.py:109-119): min-max to [0, 1]."""
    pos = np.asarray(pos)
    lo, hi = np.min(pos), np.max(pos)
    return (pos - lo) / (hi - lo)


def mask_probs(af: np.ndarray, level: int) -> np.ndarray:
    """AF-guided per-site mask probability (embedding_rag_dataset.py:527-531)."""
    return np.where(np.asarray(af) < RARE_AF_THRESHOLD, RARE_MASK_RATE, MASK_RATES[level])


def af_guided_mask(af: np.ndarray, level: int, seed: int, window_idx: int) -> np.ndarray:
    """Seeded AF-guided mask of one window, unpadded, int64 [n_sites].

    ``np.random.seed(seed * 10000 + w)`` then ``(np.random.random(n) < probs)``
    (embedding_rag_dataset.py:272-273 / :535-538, generator ``dataset.py:400``).
    The caller's global numpy RNG state is restored afterwards, as ``__getitem__``
    does (:534, :541).
    """
    probs = mask_probs(af, level)
    state = np.random.get_state()
    try:
        np.random.seed(int(seed) * 10000 + int(window_idx))
        return (np.random.random(len(probs)) < probs).astype(np.int64)
    finally:
        np.random.set_state(state)


def hwe_freqs(af_p: np.ndarray):
    p = np.asarray(af_p, dtype=np.float64)
    return (1 - p) ** 2, 2 * p * (1 - p), p ** 2
