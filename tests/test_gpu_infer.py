"""GPU tests of the imputation entry point (src/infer_embedding_rag.py): the device
post-processing kernel vs the oracle restatement of infer_embedding_rag.py:145-152
(1e-6), and an end-to-end synthetic run (retrieval + forward + post-processing +
geometry + writers) at the C5 mask sweep end points."""

import numpy as np
import pytest
import torch

from oracle import data_np

pytestmark = pytest.mark.gpu


def test_infer_post_kernel_vs_oracle():
    from src import kernels as K
    rng = np.random.default_rng(0)
    a = rng.random((3, 1030, 2)).astype(np.float32)
    b = rng.random((3, 1030, 2)).astype(np.float32)
    a /= a.sum(-1, keepdims=True)
    b /= b.sum(-1, keepdims=True)
    p1, p2, gt = K.infer_post(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda())
    o1, o2, og = data_np.infer_probs(a, b)
    np.testing.assert_allclose(p1.cpu().numpy(), o1, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(p2.cpu().numpy(), o2, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(gt.cpu().numpy(), og, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("rate", [0.1, 0.9])
def test_infer_entry_synthetic(tmp_path, rate):
    from src.infer_embedding_rag import infer
    res = infer(["--synthetic", "6", "--synthetic_windows", "2", "--synthetic_ref", "24", "-d", "64", "-l", "2",
                 "-a", "2", "-b", "4", "--k_retrieve", "3", "--window_len", "200", "--mask_rate", str(rate),
                 "-o", str(tmp_path)])
    h1, gt, mask = res["h1"], res["gt"], res["mask"]
    assert h1.shape == (400, 6) and gt.shape == (400, 6, 4) and mask.shape == (400, 6)
    assert np.isfinite(h1).all() and (h1 > 0).all() and (h1 < 1).all()
    np.testing.assert_allclose(gt.sum(-1), 1.0, rtol=1e-5)
    assert abs(mask.mean() - rate) < 0.1
    vcf = (tmp_path / "imputed.vcf").read_text().splitlines()
    body = [l for l in vcf if not l.startswith("#")]
    assert len(body) == 400 and body[0].count("\t") == 9 + 6 - 1
