"""ORACLE (test infrastructure): exact kNN over the token-resident panel index.

What it restates
----------------
The reference ranks panel haplotypes by the L2 distance between flattened
[L*D] embeddings: ``torch.cdist`` + ``topk(k, largest=False)``
(src/dataset/embedding_rag_dataset.py:390-402; FAISS ``IndexFlatL2`` in
src/dataset/embedding_rag_infer_dataset.py:176, :279-285 — same semantics).
Because ``BERTEmbedding`` is position-wise (model/embedding/bert.py:66-77),

    dist^2(q, r) = sum_l || W[tok_q,l] + A_q,l - W[tok_r,l] - A_r,l ||^2

(the positional row cancels).  All panel haplotypes share the window mask, so
only unmasked sites vary with r and ``dist^2 = C_q + sum_s Delta_q[s] * a_r[s]``
with ``a_r[s]`` the allele (0/1) of panel haplotype r at site s and
``Delta_q[s] = T_q[s, tok1] - T_q[s, tok0]``.

Canonical definition used for bit-exact parity: Delta is
quantised to a per-query power-of-two fixed-point grid (``quantize_lut``), the
distance is the exact integer ``D_q(r) = sum_s Dq_q[s] * a_r[s]`` and ties are
broken by (D, index) ascending.  The reference's fp32 cdist order equals this
order up to ties (fp32 noise picks an arbitrary member of a tied set); the
golden tests check that tie-equivalence on the reference's own outputs.
"""

from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

TOK0, TOK1, MASK_TOK = 5, 6, 4


def lut_delta(W, tok_q, dA, site_mask, tok0=TOK0, tok1=TOK1):
    """Delta_q[s] in float64 for token positions l = s + 1.

    W [V, D] fp32; tok_q [Bq, L]; dA [Bq, L, D] or None (A_q - A_r, zero when the
    query and the panel share AF); site_mask [n_sites] (1 = masked in the index).
    """
    W64 = W.astype(np.float64)
    n_sites = site_mask.shape[0]
    u = W64[tok_q[:, 1:1 + n_sites]]                       # [Bq, S, D]
    if dA is not None:
        u = u + dA[:, 1:1 + n_sites].astype(np.float64)
    t0 = ((u - W64[tok0]) ** 2).sum(-1)
    t1 = ((u - W64[tok1]) ** 2).sum(-1)
    delta = t1 - t0
    delta[:, np.asarray(site_mask).astype(bool)] = 0.0
    return delta


_LIB = None


def _oracle_lib():
    """oracle/build/liboracle.so (oracle/lut_f32.c), built on first use if absent."""
    global _LIB
    if _LIB is None:
        here = Path(__file__).resolve().parent
        so = here / "build" / "liboracle.so"
        if not so.exists() or so.stat().st_mtime < (here / "lut_f32.c").stat().st_mtime:
            subprocess.run(["make", "-s", "-C", str(here)], check=True)
        lib = ctypes.CDLL(str(so))
        lib.oracle_lut_delta_f32.restype = ctypes.c_int
        lib.oracle_lut_delta_f32.argtypes = [ctypes.c_int64] * 3 + [ctypes.c_void_p] * 4 + [ctypes.c_int64] + \
            [ctypes.c_void_p] * 2 + [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        _LIB = lib
    return _LIB


def lut_delta_f32(W, tok_q, site_mask, Aq=None, aq_period=0, Ar=None, Wp=None, tok0=TOK0, tok1=TOK1):
    """Delta_q[s] (f32 [Bq, S]) in the DEVICE's f32 arithmetic and order (oracle/lut_f32.c restates
    csrc/knn.hip lut_kernel / lut_delta_kernel), the input of the canonical quantised order.

    W [V, D] query-side token table, Wp the panel side's (default W: snvrag_knn_lut_panel);
    Aq [P, L, D] query AF-embedding offsets (row q uses Aq[q % aq_period] when aq_period > 0),
    Ar [L, D] the panel's; either may be None (the device then takes the no-offset path)."""
    c = lambda a, dt: None if a is None else np.ascontiguousarray(a, dt)
    W = c(W, np.float32)
    Wp = W if Wp is None else c(Wp, np.float32)
    tok = c(tok_q, np.int64)
    Aq, Ar = c(Aq, np.float32), c(Ar, np.float32)
    sm = c(site_mask, np.uint8)
    nq, L = tok.shape
    S = sm.shape[0]
    out = np.zeros((nq, S), np.float32)
    ptr = lambda a: None if a is None else a.ctypes.data
    rc = _oracle_lib().oracle_lut_delta_f32(nq, L, W.shape[1], ptr(tok), ptr(W), ptr(Wp), ptr(Aq), int(aq_period),
                                            ptr(Ar), ptr(sm), S, tok0, tok1, ptr(out))
    if rc:
        raise ValueError("lut_delta_f32: D must be a multiple of 4 and the window must fit L")
    return out


def quantize_lut(delta, limbs=2):
    """Per-query power-of-two scale and rint quantisation (mirrors knn.hip ``lut_kernel``).

    The exponent is the largest e with max|Delta| * 2^e <= 2**(7*limbs) - 1 (exact
    power-of-two comparisons; the device takes floor(log2(qmax / m)) and corrects it down).
    Returns (Dq int32 [Bq, S], exp2 int32 [Bq]).  |Dq| <= 2**(7*limbs) - 1.
    """
    qmax = float((1 << (7 * limbs)) - 1)
    m = np.abs(np.asarray(delta, np.float64)).max(-1)
    e = np.where(m > 0, np.floor(np.log2(qmax / np.where(m > 0, m, 1.0))), 0).astype(np.int32)
    pos = m > 0
    for _ in range(2):                     # exact: m * 2^e <= qmax < m * 2^(e+1)
        e = np.where(pos & (m * np.exp2(e + 1.0) <= qmax), e + 1, e)
        e = np.where(pos & (m * np.exp2(e * 1.0) > qmax), e - 1, e)
    e = e.astype(np.int32)
    dq = np.rint(delta * np.exp2(e)[:, None]).astype(np.int64)
    return np.clip(dq, -qmax, qmax).astype(np.int32), e


def distances(codes, dq):
    """Exact integer D[q, r] = sum_s dq[q, s] * codes[r, s] (float64 BLAS is exact here:
    every partial sum is an integer far below 2**53)."""
    S = dq.shape[1]
    return (dq.astype(np.float64) @ codes[:, :S].astype(np.float64).T).astype(np.int64)


def topk_exact(D, k):
    """(D, idx)-ascending top-k per row; pads with (-1, INT64_MAX) when N < k."""
    Bq, N = D.shape
    idx = np.full((Bq, k), -1, np.int64)
    val = np.full((Bq, k), np.iinfo(np.int64).max, np.int64)
    kk = min(k, N)
    for q in range(Bq):
        d = D[q]
        if kk < N:
            kth = np.partition(d, kk - 1)[kk - 1]
            cand = np.nonzero(d <= kth)[0]
        else:
            cand = np.arange(N)
        order = cand[np.lexsort((cand, d[cand]))][:kk]
        idx[q, :kk], val[q, :kk] = order, d[order]
    return idx, val


def knn(codes, dq, k, chunk=1 << 16):
    """Exact top-k over a panel of any size (chunked so a 1M-haplotype panel fits RAM)."""
    Bq = dq.shape[0]
    best_i = np.full((Bq, 0), -1, np.int64)
    best_d = np.full((Bq, 0), 0, np.int64)
    for r0 in range(0, codes.shape[0], chunk):
        D = distances(codes[r0:r0 + chunk], dq)
        i, d = topk_exact(D, k)
        i = np.where(i >= 0, i + r0, -1)
        ci, cd = np.concatenate([best_i, i], 1), np.concatenate([best_d, d], 1)
        keep_i = np.full((Bq, k), -1, np.int64)
        keep_d = np.full((Bq, k), np.iinfo(np.int64).max, np.int64)
        for q in range(Bq):
            ok = ci[q] >= 0
            o = np.lexsort((ci[q][ok], cd[q][ok]))[:k]
            keep_i[q, :len(o)], keep_d[q, :len(o)] = ci[q][ok][o], cd[q][ok][o]
        best_i, best_d = keep_i, keep_d
    return best_i, best_d


def merge_partials(keys, k):
    """Merge per-shard sorted (D, idx) partial lists: keys [P, Bq, k] uint64 -> [Bq, k]."""
    P, Bq, kk = keys.shape
    flat = keys.transpose(1, 0, 2).reshape(Bq, P * kk)
    return np.sort(flat, axis=1)[:, :k]


def pack_key(d, idx):
    """uint64 key = ((D + 2^30) << 32) | idx (knn.hip ``make_key``); sorts as (D, idx)."""
    return ((np.asarray(d, np.int64) + (1 << 30)).astype(np.uint64) << np.uint64(32)) | \
        np.asarray(idx, np.int64).astype(np.uint64)


def raw_genotype_knn(ref_rows, query_rows, k):
    """ORACLE of the raw-genotype window index (build_ref_db_l2.py:86-89 IndexFlatL2 over the
    flattened 0/1 genotypes): exact squared L2 = Hamming count, (D, idx)-ascending top-k."""
    R = np.asarray(ref_rows, np.int64)
    Q = np.asarray(query_rows, np.int64)
    D = (Q[:, None, :] != R[None, :, :]).sum(-1)
    return topk_exact(D, k)
