import json
import os
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "rag-snvbert_amd"
GOLDEN = Path(__file__).resolve().parent / "golden"
for p in (str(REPO), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


def load_golden(name):
    z = np.load(GOLDEN / f"{name}.npz", allow_pickle=False)
    d = {k: z[k] for k in z.files}
    if "cfg" in d:
        d["cfg"] = json.loads(str(d["cfg"]))
    return d


def golden_state_dict(cfg):
    """Synthetic weights of a golden case, keyed like the reference state_dict."""
    from src.model.foundation_model import model_state_shapes
    from src.dataset import synthetic
    shapes = model_state_shapes(cfg["vocab"], cfg["d"], cfg["layers"], cfg["heads"])
    sd = synthetic.synth_state_dict(shapes, cfg["seed"])
    assert synthetic.state_dict_digest(sd) == cfg["sd_digest"], "synthetic weights drifted from fixture"
    return sd


@pytest.fixture(scope="session")
def golden():
    return load_golden
