"""Reference checkpoints without the reference's code (SURVEY.md §5 checkpoint/resume, §8(f)3).

The reference trainer writes a pickled whole module (pretrain_with_val_optimized.py:524-552);
its inference and resume load it (infer_embedding_rag.py:93-103, train_embedding_rag.py:155-191).
``tests/golden/ref_module_tiny.pth`` is that object, written by the reference itself
(``make_golden.py pickled``: ``torch.save(model.cpu(), path)`` of a d64/L2 BERTFoundationModel with
the fwd_tiny weights); ``ref_module_tiny_sd.npz`` is the same model's ``state_dict()``.
``model.checkpoint.load_state_dict_any`` must recover that state_dict bit-exactly and in order,
through torch's weights-only unpickler with the pickled classes as inert stubs."""

import json
import os
import subprocess
import sys
from collections import OrderedDict

import numpy as np
import pytest
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
GOLD = os.path.join(ROOT, "tests", "golden")
PTH = os.path.join(GOLD, "ref_module_tiny.pth")


def _want():
    z = np.load(os.path.join(GOLD, "ref_module_tiny_sd.npz"))
    keys = json.loads(str(z["keys"]))
    return OrderedDict((k, z[f"t{i}"]) for i, k in enumerate(keys)), str(z["digest"])


def test_pickled_reference_module_to_state_dict_bit_exact():
    from src.model.checkpoint import load_state_dict_any
    before = set(sys.modules)
    sd = load_state_dict_any(PTH)
    want, digest = _want()
    assert list(sd) == list(want)
    for k, v in want.items():
        assert sd[k].dtype == torch.from_numpy(v).dtype, k
        np.testing.assert_array_equal(sd[k].numpy(), v, err_msg=k)
    # nothing of the reference was imported to read it
    new = set(sys.modules) - before
    assert not [m for m in new if m == "model" or m.startswith("model.")], sorted(new)
    # the same weights the fwd_tiny fixture was computed with
    assert digest == json.loads(str(np.load(os.path.join(GOLD, "fwd_tiny.npz"))["cfg"]))["sd_digest"]


def test_converted_state_dict_loads_strict_into_our_model():
    from src.model import build_model
    from src.model.checkpoint import load_state_dict_any
    sd = load_state_dict_any(PTH)
    m = build_model(12, 64, 2, 2)
    m.load_state_dict(sd, strict=True)
    for k, v in m.state_dict().items():
        assert torch.equal(v, sd[k]), k


@pytest.mark.parametrize("form", ["plain", "module_prefix", "state_dict_key", "trainer"])
def test_state_dict_formats(tmp_path, form):
    from src.model.checkpoint import load_state_dict_any
    want, _ = _want()
    sd = OrderedDict((k, torch.from_numpy(v)) for k, v in want.items())
    obj = {"plain": sd, "module_prefix": OrderedDict(("module." + k, v) for k, v in sd.items()),
           "state_dict_key": {"state_dict": sd, "epoch": 3}, "trainer": {"model": sd, "optim": {}, "epoch": 1}}[form]
    path = tmp_path / "ck.pt"
    torch.save(obj, path)
    got = load_state_dict_any(str(path))
    assert list(got) == list(want)
    assert all(torch.equal(got[k], sd[k]) for k in sd)


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned",))


def test_refuses_non_module_globals(tmp_path):
    from src.model.checkpoint import load_state_dict_any
    path = tmp_path / "evil.pt"
    torch.save({"x": _Evil()}, path)
    with pytest.raises(ValueError, match="refusing globals"):
        load_state_dict_any(str(path))


def test_convert_cli_writes_weights_only_state_dict(tmp_path):
    out = tmp_path / "sd.pt"
    env = dict(os.environ, PYTHONPATH=os.path.join(ROOT, "rag-snvbert_amd"))
    subprocess.run([sys.executable, "-m", "src.model.checkpoint", PTH, str(out)], check=True, env=env,
                   cwd=os.path.join(ROOT, "rag-snvbert_amd"))
    sd = torch.load(out, weights_only=True)
    want, _ = _want()
    assert list(sd) == list(want)
    assert all(np.array_equal(sd[k].numpy(), v) for k, v in want.items())
