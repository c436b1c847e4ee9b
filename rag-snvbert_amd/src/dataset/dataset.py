"""Panel/window featurisation (reference: src/dataset/dataset.py TrainDataset).

Same item contract as ``TrainDataset.__getitem__`` (dataset.py:455-582) and the
v18 override (embedding_rag_dataset.py:486-555), vectorised: the reference's
per-site Python loops over ``pos_to_idx`` become one numpy gather per field
(SURVEY.md §8f row 1).  Files: ``from_file`` needs h5py (absent in this image →
loud error); ``from_arrays`` takes the same data in memory.
"""

from __future__ import annotations

import math
from typing import Dict, List, Sequence

import numpy as np
import torch

from .utils import MASK_RATES, MAX_SEQ_LEN, mask_probs, position_normalize, sequence_padding
from .vocab import WordVocab

REF, HET, HOM, AF = 0, 1, 2, 3
GLOBAL = 5


class PanelData:
    """Population labels of the samples (dataset.py:37-99, without the POP.json side effect)."""

    def __init__(self, pop_list: Sequence[str]):
        self.pop_list = np.array(pop_list)
        self.pop_class_dict = {p: i for i, p in enumerate(np.unique(self.pop_list))}

    @classmethod
    def from_file(cls, fpath: str):
        pops = []
        with open(fpath) as f:
            for line in f:
                pops.append(line.strip().split()[2])
        return cls(pops[1:])


class Window:
    def __init__(self, start: np.ndarray, end: np.ndarray):
        self.window_info = np.stack((np.asarray(start), np.asarray(end)), axis=1)

    @classmethod
    def from_file(cls, fpath: str):
        import pandas as pd
        df = pd.read_csv(fpath, usecols=[0, 1])
        return cls(df.iloc[:, 0].astype(int).to_numpy(), df.iloc[:, 1].astype(int).to_numpy())


class TrainDataset(torch.utils.data.Dataset):
    long_fields = ["hap_1", "hap_2", "hap_1_label", "hap_2_label", "gt_label", "mask", "hap1_nomask", "hap2_nomask"]
    float_fields = ["pos", "af", "af_p", "ref", "het", "hom"]

    def __init__(self, vocab: WordVocab, vcf: np.ndarray, pos: np.ndarray, panel: PanelData, freq: np.ndarray,
                 window: Window, type_to_idx: Dict, pop_to_idx: Dict, pos_to_idx: Dict):
        self.vocab, self.vcf, self.pos = vocab, vcf, np.asarray(pos)
        self.panel, self.freq, self.window = panel, freq, window
        self.type_to_idx, self.pop_to_idx, self.pos_to_idx = type_to_idx, pop_to_idx, pos_to_idx
        self.window_count = self.window.window_info.shape[0]
        self.sample_count = self.vcf.shape[1] * self.window_count
        self._mask_rate = list(MASK_RATES)
        self._level = 0
        # vectorised pos -> freq column (replaces per-site dict lookups)
        self._freq_col = np.array([pos_to_idx[p] for p in self.pos], dtype=np.int64)

    # reference-private names kept for callers that poke at them (train_embedding_rag.py:334, :420)
    @property
    def _TrainDataset__level(self):
        return self._level

    @property
    def _TrainDataset__mask_rate(self):
        return self._mask_rate

    def __len__(self):
        return self.sample_count

    def add_level(self) -> None:
        """dataset.py:364-375."""
        self._level = min(self._level + 1, len(self._mask_rate) - 1)

    def generate_mask(self, length: int, mask_ratio: float = None, probs: np.ndarray = None) -> np.ndarray:
        """dataset.py:377-403 (probability-vector path; random-mask fallback)."""
        if probs is not None:
            return (np.random.random(length) < probs).astype(int)
        return (np.random.random(length) < self._mask_rate[self._level]).astype(int)

    def tokenize(self, seq: np.ndarray, mask: np.ndarray = None) -> np.ndarray:
        return self.vocab.tokenize(seq, mask)

    def _window_slice(self, w: int) -> slice:
        return slice(int(self.window.window_info[w, 0]), int(self.window.window_info[w, 1]))

    def _freqs(self, sl, pop_key: int):
        cols = self._freq_col[sl]
        pad = lambda v: sequence_padding(v, dtype="float")
        return dict(af=pad(self.freq[AF][GLOBAL][cols]), af_p=pad(self.freq[AF][pop_key][cols]),
                    ref=pad(self.freq[REF][pop_key][cols]), het=pad(self.freq[HET][pop_key][cols]),
                    hom=pad(self.freq[HOM][pop_key][cols]))

    def base_item(self, item: int, valid: np.ndarray = None) -> dict:
        """Unmasked fields of one (sample, window); ``valid`` selects window sites (panel-matched)."""
        sample_idx, window_idx = item // self.window_count, item % self.window_count
        sl = self._window_slice(window_idx)
        if valid is not None:
            sl = np.arange(sl.start, sl.stop)[valid]
        out = {"window_idx": window_idx}
        pop = self.panel.pop_list[sample_idx]
        h1 = np.asarray(self.vcf[sl, sample_idx, 0]).astype(np.int64)
        h2 = np.asarray(self.vcf[sl, sample_idx, 1]).astype(np.int64)
        out["hap_1_label"] = sequence_padding(h1, "int")
        out["hap_2_label"] = sequence_padding(h2, "int")
        out["gt_label"] = sequence_padding((h1 << 1) + h2, "int")
        out["hap1_nomask"], out["hap2_nomask"] = h1, h2
        out["pos"] = sequence_padding(position_normalize(self.pos[sl]), "float")
        out.update(self._freqs(sl, self.pop_to_idx[pop]))
        return out

    def __getitem__(self, item: int) -> dict:
        out = self.base_item(item)
        mask = sequence_padding(self.generate_mask(len(out["hap1_nomask"])), "int")
        out["mask"] = mask
        out["hap_1"] = self.tokenize(out["hap1_nomask"], mask)
        out["hap_2"] = self.tokenize(out["hap2_nomask"], mask)
        return self.to_tensors(out)

    def to_tensors(self, out: dict) -> dict:
        for k in self.long_fields:
            if k in out:
                out[k] = torch.as_tensor(np.asarray(out[k]), dtype=torch.long)
        for k in self.float_fields:
            if k in out:
                out[k] = torch.as_tensor(np.asarray(out[k]), dtype=torch.float32)
        return out

    @classmethod
    def from_file(cls, vocab, vcfpath, panelpath, freqpath, windowpath, typepath, poppath, pospath):
        gt, pos, t2i, p2i, pos2i = _read_inputs(vcfpath, typepath, poppath, pospath)
        return cls(vocab, gt, pos, PanelData.from_file(panelpath), np.load(freqpath),
                   Window.from_file(windowpath), t2i, p2i, pos2i)


def _read_inputs(vcfpath, typepath, poppath, pospath):
    """GT (ALT > 0 -> 1), POS and the three mapping pickles (dataset.py:190-230, :747-771).
    The pickles are the reference's own mapping files, opened as the reference does."""
    try:
        import h5py
    except ImportError as e:
        raise RuntimeError("reading the VCF/H5 inputs needs h5py (not installed here); "
                           "use from_arrays with in-memory GT/POS") from e
    import pickle
    with h5py.File(vcfpath, "r") as f:
        gt = f["calldata/GT"][:]
        pos = f["variants/POS"][:]
    gt[gt > 0] = 1
    maps = []
    for path in (typepath, poppath, pospath):
        with open(path, "rb") as fh:
            maps.append(pickle.load(fh))
    return (gt, pos, *maps)


INFER_WINDOW_LEN = 1020     # dataset.py:26


class InferDataset(torch.utils.data.Dataset):
    """Imputation featurisation (dataset.py:629-900), vectorised.

    Sites are the panel's full site list ``ori_pos`` (the keys of ``pos_to_idx``, in
    insertion order); a site absent from the target VCF is ``position_needed`` — its
    haplotype value is 0 and its mask bit 1 (the sites to impute).  Items run
    sample-major: ``item = sample * window_count + window`` over fixed windows of
    ``window_len`` sites (dataset.py:700, :818-825)."""
    long_fields = ["hap_1", "hap_2", "mask", "sample_idx", "start_idx", "end_idx", "hap1_nomask", "hap2_nomask"]
    float_fields = ["pos", "af", "af_p", "ref", "het", "hom"]

    def __init__(self, vocab: WordVocab, vcf: np.ndarray, pos: np.ndarray, panel: PanelData, freq: np.ndarray,
                 type_to_idx: Dict, pop_to_idx: Dict, pos_to_idx: Dict, window_len: int = INFER_WINDOW_LEN):
        self.vocab, self.vcf, self.pos = vocab, vcf, np.asarray(pos)
        self.panel, self.freq = panel, freq
        self.type_to_idx, self.pop_to_idx, self.pos_to_idx = type_to_idx, pop_to_idx, pos_to_idx
        self.window_len = int(window_len)
        self.ori_pos = np.array(list(pos_to_idx.keys()))
        self.position_needed = ~np.isin(self.ori_pos, self.pos, assume_unique=True)
        self.test_pos_to_idx = {p: i for i, p in enumerate(self.pos)}
        # vectorised lookups: target-VCF row of every panel site (-1 = absent) and its freq column
        self._vcf_row = np.full(len(self.ori_pos), -1, np.int64)
        if len(self.pos):
            order = np.argsort(self.pos, kind="stable")
            # last occurrence of a duplicated position, like the reference's dict (dataset.py:692)
            at = np.clip(np.searchsorted(self.pos[order], self.ori_pos, side="right") - 1, 0, len(self.pos) - 1)
            hit = self.pos[order][at] == self.ori_pos
            self._vcf_row[hit] = order[at][hit]
        self._freq_col = np.fromiter(pos_to_idx.values(), dtype=np.int64, count=len(pos_to_idx))
        self.window_count = math.ceil(self.ori_pos.shape[0] / self.window_len)
        self.sample_count = self.vcf.shape[1] * self.window_count

    def __len__(self):
        return self.sample_count

    def tokenize(self, seq: np.ndarray, mask: np.ndarray = None) -> np.ndarray:
        return self.vocab.tokenize(seq, mask)

    def window_bounds(self, w: int):
        start = self.window_len * w
        return start, min(start + self.window_len, self.ori_pos.shape[0])

    def __getitem__(self, item: int) -> dict:
        sample_idx, window_idx = item // self.window_count, item % self.window_count
        start, end = self.window_bounds(window_idx)
        out = {"sample_idx": [sample_idx], "start_idx": [start], "end_idx": [end]}
        rows = self._vcf_row[start:end]
        need = rows < 0
        h1 = np.where(need, 0, np.asarray(self.vcf[np.maximum(rows, 0), sample_idx, 0])).astype(np.int64)
        h2 = np.where(need, 0, np.asarray(self.vcf[np.maximum(rows, 0), sample_idx, 1])).astype(np.int64)
        mask = sequence_padding(need.astype(np.int64), "int")
        out["mask"] = mask
        out["hap1_nomask"], out["hap2_nomask"] = h1, h2
        out["hap_1"] = self.tokenize(h1, mask)
        out["hap_2"] = self.tokenize(h2, mask)
        out["pos"] = sequence_padding(position_normalize(self.ori_pos[start:end]), "float")
        pop_key = self.pop_to_idx[self.panel.pop_list[sample_idx]]
        cols = self._freq_col[start:end]
        pad = lambda v: sequence_padding(v, dtype="float")
        out.update(af=pad(self.freq[AF][GLOBAL][cols]), af_p=pad(self.freq[AF][pop_key][cols]),
                   ref=pad(self.freq[REF][pop_key][cols]), het=pad(self.freq[HET][pop_key][cols]),
                   hom=pad(self.freq[HOM][pop_key][cols]))
        return self.to_tensors(out)

    def to_tensors(self, out: dict) -> dict:
        return TrainDataset.to_tensors(self, out)

    @classmethod
    def from_file(cls, vocab, vcfpath, panelpath, freqpath, typepath, poppath, pospath):
        gt, pos, t2i, p2i, pos2i = _read_inputs(vcfpath, typepath, poppath, pospath)
        return cls(vocab, gt, pos, PanelData.from_file(panelpath), np.load(freqpath), t2i, p2i, pos2i)
