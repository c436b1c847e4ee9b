"""Raw-genotype window index tooling (build_ref_db_l2.py:15-98) on the host: the export writes
the reference's per-window files with the reference's transpose/flatten, the bit packing
round-trips, and the oracle (exact L2 = Hamming on 0/1 genotypes) agrees with a brute-force
float L2 over the flattened rows — the semantics of faiss.IndexFlatL2 on those rows."""

import json

import numpy as np

from oracle import knn_np


def test_build_ref_db_files_and_packing(tmp_path):
    from src.build_ref_db_l2 import main
    from src.retrieval.raw_index import flatten_window, pack_rows
    n = main(["--synthetic", "40", "--synthetic_sites", "700", "--synthetic_window", "300", "--output_dir",
              str(tmp_path)])
    assert n == 3
    from src.dataset.synthetic import make_infer_arrays
    gt = make_infer_arrays(700, 1, 40, seed=3)["ref_gt"]
    for w, (a, b) in enumerate([(0, 300), (300, 600), (600, 700)]):
        win = np.load(tmp_path / f"window_{w}.npy")
        np.testing.assert_array_equal(win, np.transpose(gt[a:b], (1, 0, 2)))
        assert np.load(tmp_path / f"window_{w}_pop.npy").shape == (40,)
        z = np.load(tmp_path / f"window_{w}.rawidx.npz")
        meta = json.loads(str(z["meta"]))
        assert meta["n_bits"] == 2 * (b - a) and meta["n"] == 40
        flat = flatten_window(gt[a:b])
        np.testing.assert_array_equal(flat, win.reshape(40, -1))
        words = z["words"].view(np.uint32)
        unpacked = np.unpackbits(words.view(np.uint8).reshape(40, -1), axis=1, bitorder="little")[:, :meta["n_bits"]]
        np.testing.assert_array_equal(unpacked, flat)
        np.testing.assert_array_equal(z["words"], pack_rows(flat))


def test_raw_oracle_equals_float_l2():
    rng = np.random.default_rng(0)
    R = (rng.random((60, 130)) < 0.3).astype(np.uint8)
    R[10] = R[3]                                        # tie
    Q = np.concatenate([R[[3, 7]], (rng.random((4, 130)) < 0.3).astype(np.uint8)])
    I, D = knn_np.raw_genotype_knn(R, Q, 8)
    L2 = ((Q[:, None, :].astype(np.float64) - R[None].astype(np.float64)) ** 2).sum(-1)
    for q in range(len(Q)):
        order = np.lexsort((np.arange(len(R)), L2[q]))[:8]
        np.testing.assert_array_equal(I[q], order)
        np.testing.assert_array_equal(D[q], L2[q][order])
    assert list(I[0][:2]) == [3, 10]
