"""The hot-path kernels of the built library stay spill-free (CPU test, no GPU).

Reads the AMDGPU code-object metadata (``NT_AMDGPU_METADATA``: ``.private_segment_fixed_size``,
``.vgpr_spill_count``) of every gfx950 code object embedded in ``lib/libsnvrag.so`` with
``llvm-readelf --notes``.  Round 2's block tail spilled 43 registers (172 B of scratch per lane, the
0.18 GB per launch of excess WRITE traffic in ``profiles/pmc_traffic.json``); DESIGN.md §4 says how
it was removed.  A spill creeping back into any kernel the bench or the train step runs fails here.
"""
import os
import re
import shutil
import struct
import subprocess
import tempfile

import pytest

LIB = os.path.join(os.path.dirname(__file__), "..", "rag-snvbert_amd", "lib", "libsnvrag.so")
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"

# (demangled-name prefix, what runs it)
HOT = [
    ("snvrag::tail_kernel<384, true, 4, 0, true, 0>", "block tail (bench roofline kernel)"),
    ("snvrag::attn32_dma<true, false, 0>", "inference attention"),
    ("snvrag::attn32_dma<false, true, 0>", "training attention forward"),
    ("snvrag::attn_bwd_dkv32", "training attention backward dK/dV"),
    ("snvrag::attn_bwd_dq32", "training attention backward dQ"),
    ("snvrag::sg_kernel<384, 0, 0, false, 8, false>", "QKV stream GEMM"),
    ("snvrag::mlp_kernel<384, true, 1, false>", "hap-head fused MLP"),
    ("snvrag::mlp_kernel<384, false, 0, true>", "af_adapter fused MLP with the AF gate in its prologue"),
    ("snvrag::sg_kernel<768, 0, 1, false, 4, true>", "rag fusion cat GEMM"),
    ("snvrag::g3_kernel<4, 0, 0>", "training wide-row GEMM"),
    ("snvrag::g3_kernel<7, 0, 0>", "training wide-row GEMM (M = 49 440)"),
    ("snvrag::g3_kernel<6, 0, 1>", "rag fusion K = 4D projection + LN / MAF tail (bench M)"),
    ("snvrag::g3_kernel<7, 0, 1>", "rag fusion K = 4D projection + LN / MAF tail"),
    ("snvrag::tailw_kernel<0>", "wide-row block tail (bench roofline kernel)"),
    ("snvrag::dw_dma_kernel", "training dW"),
    ("snvrag::scan2_kernel<16, 2, 0>", "kNN panel scan"),
    # (bf16 template arguments: c++filt leaves these names mangled)
    ("_ZN6snvrag13ln_bwd_kernel", "training LayerNorm backward (N <= 512)"),
    ("_ZN6snvrag16ln_bwd_pf_kernel", "training LayerNorm backward (N > 512)"),
    ("_ZN6snvrag19ln_fwd_train_kernel", "training LayerNorm forward"),
]


def _code_objects(data: bytes):
    """gfx ELF images embedded in the host library's offload section."""
    out, i = [], 0
    while True:
        j = data.find(b"\x7fELF", i + 1)
        if j < 0:
            return out
        i = j
        if data[j + 4] != 2 or struct.unpack_from("<H", data, j + 18)[0] != 0xE0:   # ELF64, EM_AMDGPU
            continue
        shoff = struct.unpack_from("<Q", data, j + 0x28)[0]
        shentsize, shnum = struct.unpack_from("<HH", data, j + 0x3A)
        out.append(data[j:j + shoff + shentsize * shnum])


def _kernel_resources():
    res = {}
    with open(LIB, "rb") as f:
        objs = _code_objects(f.read())
    with tempfile.TemporaryDirectory() as td:
        for n, co in enumerate(objs):
            p = os.path.join(td, f"co{n}.o")
            with open(p, "wb") as f:
                f.write(co)
            notes = subprocess.run([READELF, "--notes", p], capture_output=True, text=True, check=True).stdout
            for chunk in re.split(r"\n  - \.", notes)[1:]:
                name = re.search(r"\n    \.name:\s+(\S+)", chunk)
                scratch = re.search(r"\n    \.private_segment_fixed_size:\s+(\d+)", chunk)
                spills = re.search(r"\n    \.vgpr_spill_count:\s+(\d+)", chunk)
                if name and scratch:
                    res[name.group(1)] = (int(scratch.group(1)), int(spills.group(1)) if spills else 0)
    demangled = subprocess.run(["c++filt"], input="\n".join(res), capture_output=True, text=True).stdout.split("\n")
    return {d[5:] if d.startswith("void ") else d: v for d, v in zip(demangled, res.values())}


@pytest.mark.skipif(not (os.path.exists(LIB) and os.path.exists(READELF) and shutil.which("c++filt")),
                    reason="library not built or ROCm llvm-readelf absent")
def test_hot_kernels_are_spill_free():
    res = _kernel_resources()
    assert len(res) > 100, "kernel metadata not found in the library"
    for prefix, what in HOT:
        hits = {k: v for k, v in res.items() if k.startswith(prefix)}
        assert hits, f"{prefix} ({what}) not in the library"
        for k, (scratch, spills) in hits.items():
            assert scratch == 0 and spills == 0, f"{k} ({what}): {scratch} B scratch/lane, {spills} VGPR spills"
