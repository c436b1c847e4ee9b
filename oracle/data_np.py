"""ORACLE (test infrastructure): data-contract restatements.

  tokenize           src/dataset/dataset.py:597-625 + vocab.py:153-170
  sequence_padding   src/dataset/utils.py:121-132
  position_normalize src/dataset/utils.py:109-119
  AF-guided mask     src/dataset/embedding_rag_dataset.py:527-544 (generator dataset.py:396-400)
  infer post-process src/infer_embedding_rag.py:145-152 (probabilities) and :166-203 (geometry)
"""

from __future__ import annotations

import numpy as np

MAX_SEQ_LEN = 1030


def tokenize(seq, mask, stoi, sos=2, eos=3, pad=0, unk=1, mask_tok=4, seq_len=MAX_SEQ_LEN):
    seq = np.asarray(seq)
    rows = seq.reshape(-1, seq.shape[-1])
    out = np.full((rows.shape[0], seq_len), pad, np.int64)
    for i, r in enumerate(rows):
        t = [sos] + [stoi.get(int(v), unk) for v in r] + [eos]
        t = t[:seq_len]
        out[i, :len(t)] = t
    if mask is not None:
        out = np.where(np.asarray(mask).astype(bool), mask_tok, out)
    return out.reshape(seq.shape[:-1] + (seq_len,))


def sequence_padding(seq, dtype="int", seq_len=MAX_SEQ_LEN):
    pad = 0 if dtype == "int" else 0.0
    pre = np.array([pad])
    post = np.array([pad for _ in range(seq_len - len(seq) - 1)])
    return np.concatenate((pre, np.asarray(seq), post))


def position_normalize(pos):
    pos = np.asarray(pos)
    return (pos - pos.min()) / (pos.max() - pos.min())


def af_mask(af, rate, seed, w, rare_thr=0.05, rare_rate=0.7):
    probs = np.where(np.asarray(af) < rare_thr, rare_rate, rate)
    st = np.random.get_state()
    np.random.seed(seed * 10000 + w)
    m = (np.random.random(len(probs)) < probs).astype(int)
    np.random.set_state(st)
    return m


def infer_probs(probs_h1, probs_h2):
    """infer_embedding_rag.py:145-152: softmax applied AGAIN to the head's probabilities."""
    def sm(x):
        e = np.exp(x - x.max(-1, keepdims=True))
        return e / e.sum(-1, keepdims=True)
    p1, p2 = sm(probs_h1)[..., 1], sm(probs_h2)[..., 1]
    gt = np.stack([(1 - p1) * (1 - p2), (1 - p1) * p2, p1 * (1 - p2), p1 * p2], -1)
    return p1, p2, gt


def infer_geometry(h1, h2, gt, mask, n_windows, n_variants, window_len):
    """infer_embedding_rag.py:166-203: slice [1, 1+window_len), [W,S,L] -> [W*L, S], fit to n_variants."""
    h1, h2 = h1[:, 1:1 + window_len], h2[:, 1:1 + window_len]
    gt, mask = gt[:, 1:1 + window_len, :], mask[:, 1:1 + window_len]
    S = h1.shape[0] // n_windows
    L = h1.shape[1]
    h1 = h1.reshape(n_windows, S, L).transpose(0, 2, 1).reshape(-1, S)
    h2 = h2.reshape(n_windows, S, L).transpose(0, 2, 1).reshape(-1, S)
    gt = gt.reshape(n_windows, S, L, 4).transpose(0, 2, 1, 3).reshape(-1, S, 4)
    mask = mask.reshape(n_windows, S, L).transpose(0, 2, 1).reshape(-1, S)
    if h1.shape[0] >= n_variants:
        return h1[:n_variants], h2[:n_variants], gt[:n_variants], mask[:n_variants]
    pad = n_variants - h1.shape[0]
    return (np.pad(h1, ((0, pad), (0, 0))), np.pad(h2, ((0, pad), (0, 0))),
            np.pad(gt, ((0, pad), (0, 0), (0, 0))), np.pad(mask, ((0, pad), (0, 0))))
