"""Shared kNN test helpers: LUT fragment decoding and seeded random cases."""

import numpy as np
import torch


def decode_lut(lut: torch.Tensor, nq: int, n_sites_pad: int, limbs: int) -> np.ndarray:
    """Inverse of the fragment layout [qt][limb][ks][lane][16] -> int32 dq[q, s] (csrc/knn.hip lut_kernel)."""
    KS = n_sites_pad // 64
    nqt = (nq + 15) // 16
    b = lut.cpu().numpy().view(np.int8)[:nqt * limbs * KS * 1024]
    b = b.reshape(nqt, limbs, KS, 4, 16, 16)                                   # [qt][limb][ks][g][li][j]
    b = b.transpose(0, 4, 1, 2, 3, 5).reshape(nqt * 16, limbs, n_sites_pad).astype(np.int32)
    dq = b[:, 0] * 128 + b[:, 1] if limbs == 2 else b[:, 0]
    return dq[:nq]


def lut_wide_flag(lut: torch.Tensor, nq: int, n_sites_pad: int) -> int:
    """The 2-limb LUT's 'some query needs two limbs' flag (0 = the scan ran the reduced one-limb body)."""
    nqt, KS = (nq + 15) // 16, n_sites_pad // 64
    return int(lut.cpu().numpy().view(np.int8)[nqt * 3 * KS * 1024 + nqt * 64:][:4].view(np.int32)[0])


def rand_case(n_ref, n_sites, nq, seed, tie_heavy=False, D=64):
    """Random panel + queries copied from panel rows with 5 % flips; query tokens over L = 1030
    (``tie_heavy``: half the panel identical, aligned masks; otherwise a few extra query-masked sites)."""
    rng = np.random.default_rng(seed)
    W = rng.standard_normal((12, D)).astype(np.float32)
    af = rng.beta(0.3, 3.0, n_sites)
    panel = (rng.random((n_ref, n_sites)) < af).astype(np.uint8)
    if tie_heavy:
        panel[: n_ref // 2] = panel[0]
    q_alle = panel[rng.integers(0, n_ref, nq)] ^ (rng.random((nq, n_sites)) < 0.05)
    site_mask = (rng.random(n_sites) < 0.4).astype(np.uint8)
    L = 1030
    tok = np.zeros((nq, L), np.int64)
    tok[:, 0] = 2
    tok[:, 1:1 + n_sites] = np.where(site_mask[None] == 1, 4, 5 + q_alle)
    tok[:, 1 + n_sites] = 3
    if not tie_heavy:   # a few query positions masked where the panel is not (misaligned masks)
        tok[:, 1:1 + n_sites][:, rng.random(n_sites) < 0.05] = 4
    return W, panel, site_mask, tok
