"""Checkpoints written by the reference, read without running any of its code.

The reference saves a trained model as a PICKLED WHOLE MODULE — ``torch.save(self.model.cpu(),
path)`` (pretrain_with_val_optimized.py:524-552) — and its inference loads it back as the model
object itself (``model = checkpoint``, infer_embedding_rag.py:93-103); its training resume accepts
that, a plain state_dict or ``{'state_dict': ...}`` with optional ``module.`` prefixes
(train_embedding_rag.py:155-191).  A pickled module names the reference's classes
(``model.foundation_model.BERTFoundationModel``, ``model.bert.BERTWithEmbeddingRAG``, ...), which do
not exist here, and unpickling it with the plain loader would import and run whatever those
names resolve to.

``load_state_dict_any`` reads every one of those formats with torch's weights-only unpickler (the
restricted ``pickle.Unpickler`` torch ships: only allow-listed globals, tensor rebuilds from the
archive's storages, no REDUCE of anything else).  The module classes a pickled module names are
allow-listed as INERT STUBS: ``_ModuleRecord`` subclasses created here under each class's dotted
name, which record the state pickle hands them (``_parameters`` / ``_buffers`` / ``_modules``)
and nothing else — no reference (or torch.nn) class is imported or executed.  The record tree is
then flattened exactly like ``nn.Module.state_dict`` (None parameters skipped, non-persistent
buffers dropped), giving the reference's key layout, which is ours (``BERTFoundationModel``).

Only class names under ``model.``, ``src.model.``, ``__main__.``, ``torch.nn.modules.`` and
``torch.nn.parallel.`` may be stubbed; any other non-default global in the file is refused.

    python -m src.model.checkpoint IN.pth OUT.pt   # convert to a weights_only state_dict file
"""
from __future__ import annotations

import sys
from collections import OrderedDict
from typing import Dict

import torch

STUB_PREFIXES = ("model.", "src.model.", "__main__.", "torch.nn.modules.", "torch.nn.parallel.")


class _ModuleRecord:
    """Inert stand-in for a pickled module class: pickle's BUILD step stores the module's
    ``__dict__`` here (no ``__setstate__``, so no code of the original class runs)."""
    _qualname = "?"

    def __repr__(self):
        return f"<record of {self._qualname}>"


def _stub(name: str):
    return type(name.rsplit(".", 1)[-1], (_ModuleRecord,), {"_qualname": name, "__module__": __name__})


def _flatten(rec, prefix: str, out: Dict[str, torch.Tensor]) -> None:
    """nn.Module.state_dict order: own parameters, own persistent buffers, then children."""
    d = rec.__dict__
    for k, v in (d.get("_parameters") or {}).items():
        if v is not None:
            out[prefix + k] = v.detach() if isinstance(v, torch.Tensor) else v
    skip = d.get("_non_persistent_buffers_set") or set()
    for k, v in (d.get("_buffers") or {}).items():
        if v is not None and k not in skip:
            out[prefix + k] = v
    for k, child in (d.get("_modules") or {}).items():
        if child is not None:
            if not isinstance(child, _ModuleRecord):
                raise ValueError(f"submodule {prefix + k} is a {type(child).__name__}, not a module record")
            _flatten(child, prefix + k + ".", out)


def _strip_module(sd: Dict[str, torch.Tensor]) -> "OrderedDict[str, torch.Tensor]":
    # DataParallel prefix (train_embedding_rag.py:182-186, infer_embedding_rag.py:97-98)
    return OrderedDict((k[7:] if k.startswith("module.") else k, v) for k, v in sd.items())


def load_state_dict_any(path: str) -> "OrderedDict[str, torch.Tensor]":
    """state_dict (CPU tensors) from a reference pickled-module checkpoint, a plain state_dict,
    ``{'state_dict': sd}`` or this package's trainer checkpoint (``{'model': sd, ...}``)."""
    unsafe = torch.serialization.get_unsafe_globals_in_checkpoint(path)
    bad = [g for g in unsafe if not g.startswith(STUB_PREFIXES)]
    if bad:
        raise ValueError(f"{path}: refusing globals that are not module classes: {sorted(bad)}")
    stubs = [(_stub(g), g) for g in sorted(unsafe)]
    with torch.serialization.safe_globals(stubs):
        obj = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(obj, _ModuleRecord):
        sd: Dict[str, torch.Tensor] = OrderedDict()
        _flatten(obj, "", sd)
        return _strip_module(sd)
    if isinstance(obj, dict):
        for key in ("model", "state_dict"):
            if key in obj and isinstance(obj[key], dict):
                obj = obj[key]
                break
        if any(isinstance(v, _ModuleRecord) for v in obj.values()):
            raise ValueError(f"{path}: a dict holding module objects is not a state_dict")
        return _strip_module(obj)
    raise ValueError(f"{path}: unknown checkpoint format {type(obj).__name__}")


def main(argv=None) -> None:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) != 2:
        raise SystemExit("usage: python -m src.model.checkpoint IN.pth OUT.pt")
    sd = load_state_dict_any(argv[0])
    torch.save(sd, argv[1])
    print(f"{argv[0]}: {len(sd)} tensors -> {argv[1]}")


if __name__ == "__main__":
    main()
