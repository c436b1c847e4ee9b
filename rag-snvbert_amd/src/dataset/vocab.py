"""Vocabulary contract of the reference.

Token ids follow ``src/dataset/vocab.py:91-98`` (specials) and ``:122-151``
(``WordVocab``: alleles first, then population labels in first-seen order):

    <pad>=0 <unk>=1 <sos>=2 <eos>=3 <mask>=4, allele 0 -> 5, allele 1 -> 6, pops 7+

``to_seq`` is ``vocab.py:153-170``: ``[<sos>] + ids + [<eos>]`` then pad /
truncate to ``seq_len``.  The vectorised :meth:`WordVocab.tokenize` replaces the
per-haplotype list comprehension of ``dataset.py:597-625`` with one numpy
gather; same output.
"""

from __future__ import annotations

from collections import Counter
from typing import Iterable, List, Sequence

import numpy as np

PAD, UNK, SOS, EOS, MASK = 0, 1, 2, 3, 4
MAX_SEQ_LEN = 1030


class Vocab:
    def __init__(self, counter: Counter):
        self.pad_index, self.unk_index, self.sos_index = PAD, UNK, SOS
        self.eos_index, self.mask_index = EOS, MASK
        self.itos: List = ["<pad>", "<unk>", "<sos>", "<eos>", "<mask>"]
        for tok in list(self.itos):
            counter.pop(tok, None)
        for word in counter:          # dict order == first insertion (vocab.py:54-58)
            self.itos.append(word)
        self.stoi = {tok: i for i, tok in enumerate(self.itos)}

    def __len__(self) -> int:
        return len(self.itos)


class WordVocab(Vocab):
    """``WordVocab(pop_vocab)``: Counter([0, 1]) then the population labels."""

    def __init__(self, pop_vocab: Sequence[str]):
        merged = Counter()
        merged.update(Counter([0, 1]))
        merged.update(Counter(pop_vocab))
        super().__init__(merged)

    def to_seq(self, sentence: Iterable, seq_len: int | None = None,
               with_sos: bool = False, with_len: bool = False):
        seq = [self.stoi.get(w, self.unk_index) for w in sentence]
        if with_sos:
            seq = [self.sos_index] + seq + [self.eos_index]
        origin = len(seq)
        if seq_len is not None:
            seq = (seq + [self.pad_index] * (seq_len - len(seq)))[:seq_len]
        return (seq, origin) if with_len else seq

    # ----------------------------------------------------------------- #
    def allele_lut(self) -> np.ndarray:
        """int64 lookup genotype value -> token id for values -1..255 (offset +1)."""
        lut = np.full(257, self.unk_index, dtype=np.int64)
        for v in range(-1, 256):
            lut[v + 1] = self.stoi.get(v, self.unk_index)
        return lut

    def tokenize(self, seq: np.ndarray, mask: np.ndarray | None = None,
                 seq_len: int = MAX_SEQ_LEN) -> np.ndarray:
        """Vectorised ``TrainDataset.tokenize`` (dataset.py:597-625).

        seq  : int [..., n] genotype values (alleles)
        mask : int [seq_len] or [..., seq_len] padded mask, 1 = replace by <mask>
        returns int64 [..., seq_len]
        """
        seq = np.asarray(seq)
        lead, n = seq.shape[:-1], seq.shape[-1]
        out = np.full(lead + (seq_len,), self.pad_index, dtype=np.int64)
        body = self.allele_lut()[np.clip(seq.astype(np.int64), -1, 255) + 1]
        toks = np.concatenate([np.full(lead + (1,), self.sos_index, np.int64), body,
                               np.full(lead + (1,), self.eos_index, np.int64)], axis=-1)
        m = min(seq_len, n + 2)
        out[..., :m] = toks[..., :m]
        if mask is not None:
            out = np.where(np.asarray(mask).astype(bool), self.mask_index, out)
        return out
