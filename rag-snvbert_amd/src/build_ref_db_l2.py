"""Offline raw-genotype reference index per window (reference: build_ref_db_l2.py:15-114).

    python -m src.build_ref_db_l2 --ref_vcf panel.h5 --ref_panel panel.txt --window_csv window.csv \\
        --output_dir ref_db/

Per window: ``window_{w}.npy`` (samples, window_len, 2) genotypes, ``window_{w}_pop.npy``
population labels and ``window_{w}.rawidx.npz`` — the bit-packed rows of the
HBM-resident exact-L2 (= Hamming on 0/1 genotypes) index that replaces the reference's
``window_{w}.faiss`` (retrieval/raw_index.py; search with ``raw_index.load_window``).
``--synthetic N`` writes an in-memory synthetic panel of N samples instead of reading
files (h5py / scikit-allel are not installed in this image).
"""

from __future__ import annotations

import argparse
import sys

import numpy as np


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="raw-genotype window index (MI355X)")
    p.add_argument("--ref_vcf", type=str, default=None, help="reference HDF5 (calldata/GT, variants/POS)")
    p.add_argument("--ref_panel", type=str, default=None, help="panel file (population labels)")
    p.add_argument("--window_csv", type=str, default=None, help="window.csv shared with the target data")
    p.add_argument("--output_dir", type=str, required=True)
    p.add_argument("--synthetic", type=int, default=0, help="synthetic panel samples (no input files)")
    p.add_argument("--synthetic_sites", type=int, default=2040)
    p.add_argument("--synthetic_window", type=int, default=1020)
    return p.parse_args(argv)


def main(argv=None) -> int:
    from .retrieval.raw_index import build_ref_db
    args = parse_args(argv)
    if args.synthetic:
        from .dataset.synthetic import POPS, make_infer_arrays
        a = make_infer_arrays(args.synthetic_sites, 1, args.synthetic, seed=3)
        gt, pops = a["ref_gt"], [POPS[i % 5] for i in range(args.synthetic)]
        n = gt.shape[0]
        bounds = np.array([[s, min(s + args.synthetic_window, n)] for s in range(0, n, args.synthetic_window)])
    else:
        from .dataset.dataset import PanelData, Window
        try:
            import h5py
        except ImportError as e:
            raise SystemExit("reading the reference HDF5 needs h5py (not installed here); use --synthetic N") from e
        with h5py.File(args.ref_vcf, "r") as f:
            gt = f["calldata/GT"][:]
        pops = PanelData.from_file(args.ref_panel).pop_list
        bounds = Window.from_file(args.window_csv).window_info
    n_windows = build_ref_db(gt, pops, bounds, args.output_dir)
    print(f"[build_ref_db_l2] Done! {n_windows} windows saved to {args.output_dir}", flush=True)
    return n_windows


if __name__ == "__main__":
    main(sys.argv[1:])
