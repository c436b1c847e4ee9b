"""Raw-genotype window index (reference: build_ref_db_l2.py:15-98, test_faiss_intersect.py:130-205).

The reference's offline tool stores, per window of window.csv, the panel samples'
genotypes ``window_{w}.npy`` (samples, window_len, 2), their populations
``window_{w}_pop.npy`` and a ``faiss.IndexFlatL2`` over the flattened
(samples, window_len * 2) 0/1 float rows (``window_{w}.faiss``).  Exact L2 on 0/1
vectors is the Hamming distance, so here a window's index is the rows bit-packed
(32 genotypes per word, word-major so the GPU scan reads coalesced lines) —
``window_{w}.rawidx.npz`` — searched on the device by popcount (csrc/rawdb.hip) with the
kNN's exact (distance, row) top-k.  ``search`` returns what ``IndexFlatL2.search``
returns: squared L2 distances (float32) and int64 row ids.
"""

from __future__ import annotations

import json
import os
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from .. import kernels as K


def pack_rows(bits: np.ndarray) -> np.ndarray:
    """0/1 [n, B] -> int32 [n, ceil(B / 32)]: bit b of row r at word b // 32, bit b % 32."""
    bits = np.asarray(bits).astype(np.uint8)
    n, B = bits.shape
    nw = (B + 31) // 32
    padded = np.zeros((n, nw * 32), np.uint8)
    padded[:, :B] = bits
    by = np.packbits(padded.reshape(n, nw * 4, 8), axis=-1, bitorder="little").reshape(n, nw * 4)
    return by.view("<u4").astype(np.uint32).view(np.int32)


def flatten_window(gt_window: np.ndarray) -> np.ndarray:
    """(window_len, samples, 2) GT -> (samples, window_len * 2) 0/1, the reference's
    transpose + reshape (build_ref_db_l2.py:72-88), ALT > 0 -> 1 (:52)."""
    g = np.asarray(gt_window)
    g = (g > 0).astype(np.uint8)
    return np.transpose(g, (1, 0, 2)).reshape(g.shape[1], -1)


class RawGenotypeIndex:
    """One window's raw-genotype index resident in HBM."""

    def __init__(self, words: np.ndarray, n_bits: int, device):
        self.n, self.nw = words.shape
        self.n_bits = int(n_bits)
        self.codes_wm = torch.from_numpy(np.ascontiguousarray(words.T)).to(device)

    @classmethod
    def from_genotypes(cls, gt_window: np.ndarray, device) -> "RawGenotypeIndex":
        flat = flatten_window(gt_window)
        return cls(pack_rows(flat), flat.shape[1], device)

    def search(self, queries: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
        """queries: (nq, window_len * 2) 0/1 rows (or (nq, window_len, 2)) -> (D f32 [nq, k], I int64 [nq, k]);
        rows beyond the panel size pad with (inf, -1) like faiss."""
        q = np.asarray(queries).reshape(len(queries), -1)
        if q.shape[1] != self.n_bits:
            raise ValueError(f"query rows have {q.shape[1]} genotypes, the index {self.n_bits}")
        kk = min(k, 32)
        if k > 32:
            raise ValueError("k <= 32")
        qw = torch.from_numpy(pack_rows(q)).to(self.codes_wm.device)
        keys = K.hamming_topk(self.codes_wm, qw, kk).cpu().numpy().view(np.uint64)
        I = (keys & np.uint64(0xFFFFFFFF)).astype(np.int64)
        D = ((keys >> np.uint64(32)).astype(np.int64) - (1 << 30)).astype(np.float32)
        empty = I >= self.n
        I[empty], D[empty] = -1, np.inf
        return D, I


def build_ref_db(gt: np.ndarray, pop_list: Sequence[str], window_bounds: np.ndarray, output_dir: str) -> int:
    """build_ref_db_l2.py:15-98 over in-memory arrays: GT (variants, samples, 2), the panel's
    population labels and window.csv's [start, end) rows.  Writes window_{w}.npy (int8
    (samples, window_len, 2)), window_{w}_pop.npy and window_{w}.rawidx.npz per window.
    Returns the number of windows."""
    gt = np.asarray(gt)
    if len(pop_list) != gt.shape[1]:
        raise ValueError(f"Panel sample count ({len(pop_list)}) != VCF sample count ({gt.shape[1]})")
    os.makedirs(output_dir, exist_ok=True)
    bounds = np.asarray(window_bounds)
    for w, (a, b) in enumerate(bounds):
        sub = (gt[int(a):int(b)] > 0).astype(np.int8)
        np.save(os.path.join(output_dir, f"window_{w}.npy"), np.transpose(sub, (1, 0, 2)))
        np.save(os.path.join(output_dir, f"window_{w}_pop.npy"), np.asarray(pop_list))
        flat = flatten_window(sub)
        np.savez(os.path.join(output_dir, f"window_{w}.rawidx.npz"), words=pack_rows(flat),
                 meta=np.array(json.dumps(dict(n_bits=int(flat.shape[1]), n=int(flat.shape[0]), start=int(a),
                                               end=int(b)))))
    return len(bounds)


def load_window(output_dir: str, w: int, device) -> RawGenotypeIndex:
    z = np.load(os.path.join(output_dir, f"window_{w}.rawidx.npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    return RawGenotypeIndex(z["words"], meta["n_bits"], device)
