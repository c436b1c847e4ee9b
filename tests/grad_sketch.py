"""Compact, deterministic sketches of large gradient tensors (test infrastructure).

The v18-size training fixture (d384 / L12 / H12, ~26 M parameters) cannot be committed as full
gradients (~100 MB).  Per parameter it stores instead:

  gn:<name>  the Frobenius norm of the reference gradient (float64);
  gp:<name>  NPROJ projections <g, v_j> on pseudo-random Gaussian vectors v_j seeded by the
             parameter's name (E <g - r, v>^2 = |g - r|^2, so the projections of a difference
             estimate its norm: with 16 of them the ratio is within ~+-35 % at 2 sigma);
  gs:<name>  the values at NSAMP fixed pseudo-random positions (or all of them for small tensors).

``compare`` turns a candidate gradient into (estimated relative error, sampled relative error,
sampled cosine) against such a sketch.  Used by tests/golden/make_train_golden.py (generation)
and tests/test_gpu_train.py (check).
"""

from __future__ import annotations

import zlib

import numpy as np

NPROJ = 16
NSAMP = 2048


def _rng(name: str) -> np.random.Generator:
    return np.random.default_rng([zlib.crc32(name.encode()) & 0xFFFFFFFF, 0x5E7C])


def positions(name: str, n: int) -> np.ndarray:
    if n <= NSAMP:
        return np.arange(n)
    return np.sort(_rng(name + "#pos").choice(n, NSAMP, replace=False))


def projections(name: str, g: np.ndarray) -> np.ndarray:
    flat = np.asarray(g, np.float64).reshape(-1)
    rng = _rng(name)
    out = np.empty(NPROJ, np.float64)
    for j in range(NPROJ):
        v = rng.standard_normal(flat.size, dtype=np.float32)
        out[j] = float(np.dot(flat, v.astype(np.float64)))
    return out


def sketch(name: str, g: np.ndarray) -> dict:
    flat = np.asarray(g, np.float32).reshape(-1)
    return {f"gn:{name}": np.float64(np.linalg.norm(flat.astype(np.float64))),
            f"gp:{name}": projections(name, flat),
            f"gs:{name}": flat[positions(name, flat.size)].copy()}


def names(fixture) -> list:
    return [k[3:] for k in fixture if k.startswith("gn:")]


def compare(name: str, g: np.ndarray, fixture) -> tuple:
    """(estimated |g - r| / |r| from the projections, sampled-element relative error, sampled cosine)."""
    flat = np.asarray(g, np.float32).reshape(-1)
    rn = float(fixture[f"gn:{name}"])
    dp = projections(name, flat) - np.asarray(fixture[f"gp:{name}"])
    est = float(np.sqrt(np.mean(dp ** 2))) / max(rn, 1e-30)
    s = flat[positions(name, flat.size)].astype(np.float64)
    r = np.asarray(fixture[f"gs:{name}"], np.float64)
    rel_s = float(np.linalg.norm(s - r) / max(np.linalg.norm(r), 1e-30))
    cos = float(np.dot(s, r) / max(np.linalg.norm(s) * np.linalg.norm(r), 1e-30))
    return est, rel_s, cos
