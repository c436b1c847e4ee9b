"""ctypes binding of ``lib/libsnvrag.so`` (C ABI declared in ``include/snvrag.h``).

The library is built in-tree (``make -C rag-snvbert_amd``) and loaded from
``rag-snvbert_amd/lib``.  There is no CPU fallback anywhere in the product path:
if the library or a GPU is missing, every operator raises.

Tensor arguments are torch tensors living on the current HIP device; only their
``data_ptr()`` crosses the boundary, together with the current HIP stream.
"""

from __future__ import annotations

import ctypes as C
import os
from pathlib import Path
from typing import Optional

import torch

PKG_DIR = Path(__file__).resolve().parents[1]
LIB_PATH = Path(os.environ.get("SNVRAG_LIB", PKG_DIR / "lib" / "libsnvrag.so"))

F32, BF16 = 0, 1
ACT_NONE, ACT_GELU, ACT_LRELU, ACT_SIGMOID = 0, 1, 2, 3
ABI_VERSION = 28

vp, i64, i32, f32, sz = C.c_void_p, C.c_int64, C.c_int32, C.c_float, C.c_size_t


class DeriveJob(C.Structure):
    _fields_ = [("kind", i32), ("nparts", i32), ("rows", i64), ("cols", i64), ("dst_ld", i64),
                ("piece0", i64), ("pieces", i64), ("part_rows", i64 * 4), ("rs", i64 * 4), ("cs", i64 * 4),
                ("src", vp * 4), ("dst", vp)]


class Epilogue(C.Structure):
    _fields_ = [("bias", vp), ("row1", vp), ("row1_stride", i64), ("col1", vp),
                ("row2", vp), ("row2_stride", i64), ("col2", vp), ("row_period", i64),
                ("act", C.c_int), ("slope", f32), ("resid", vp), ("ld_resid", i64),
                ("ln_g", vp), ("ln_b", vp), ("ln_eps", f32), ("ln_act", C.c_int),
                ("post_base", vp), ("ld_post", i64), ("post_scale", f32),
                ("post_af", vp), ("post_af_period", i64), ("post_maf", C.c_int),
                ("stats_out", vp)]


class RowNormS(C.Structure):
    _fields_ = [("stats", vp), ("n_parts", C.c_int), ("dim", i64), ("eps", f32), ("c1", vp)]


class LnPost(C.Structure):
    _fields_ = [("base", vp), ("ld_base", i64), ("scale", f32), ("af", vp),
                ("af_period", i64), ("maf_weight", C.c_int), ("act", C.c_int)]


class PosfeatW(C.Structure):
    _fields_ = [(n, vp) for n in ("c1_w", "c1_b", "c2_w", "c2_b", "c3_w", "c3_b",
                                  "bn1_w", "bn1_b", "bn1_rm", "bn1_rv",
                                  "bn2_w", "bn2_b", "bn2_rm", "bn2_rv")] + [("bn_eps", f32)]


class AfGateW(C.Structure):
    _fields_ = [(n, vp) for n in ("g1_w", "g1_b", "g2_w", "g2_b", "j_w", "j_b", "ln_w", "ln_b")] + \
               [("res_scale", f32)]


class GtW(C.Structure):
    _fields_ = [(n, vp) for n in ("f_w", "f_b", "n_w", "n_b", "w1", "b1", "ln_w", "ln_b",
                                  "w2", "b2", "c_w", "c_b")]


class AdamS(C.Structure):
    _fields_ = [("lr", f32), ("beta1", f32), ("beta2", f32), ("eps", f32), ("weight_decay", f32),
                ("grad_scale", f32), ("max_norm", f32), ("step", C.c_int)]


class LayerW(C.Structure):
    _fields_ = [(n, vp) for n in ("w_qkv", "b_qkv", "w_o", "b_o", "ln1_g", "ln1_b", "w1", "b1",
                                  "lnf_g", "lnf_b", "w2", "b2", "ln2_g", "ln2_b", "w2g", "b2g", "c2g")] + [("q_scale", f32)] + \
        [("ffn_v", vp), ("tail_w", vp), ("qkv_pw", vp), ("qkv_sg", vp)]


_SIGS = {
    "snvrag_abi_version": ([], C.c_int),
    "snvrag_last_error": ([], C.c_char_p),
    "snvrag_device_info": ([C.c_int, C.c_char_p, C.c_int], C.c_int),
    "snvrag_set_option": ([C.c_char_p, i64], C.c_int),
    "snvrag_get_option": ([C.c_char_p, C.POINTER(i64)], C.c_int),
    "snvrag_linear": ([C.c_int, C.c_int, i64, i64, i64, vp, i64, vp, i64, vp, i64, C.POINTER(Epilogue), vp], C.c_int),
    "snvrag_linear_ex": ([C.c_int, C.c_int, i64, i64, i64, vp, i64, vp, i64, vp, i64, C.POINTER(Epilogue),
                          C.POINTER(RowNormS), vp], C.c_int),
    "snvrag_layernorm": ([C.c_int, C.c_int, i64, i64, vp, i64, vp, i64, vp, vp, f32, vp, i64,
                          C.POINTER(LnPost), vp], C.c_int),
    "snvrag_attention": ([C.c_int, i64, i64, C.c_int, C.c_int, vp, i64, vp, i64, f32, vp], C.c_int),
    "snvrag_attention_fallbacks": ([C.c_int], C.c_int),
    "snvrag_af_features": ([C.c_int, i64, vp, vp, C.c_int, vp, vp], C.c_int),
    "snvrag_embed_tokens": ([C.c_int, i64, i64, i64, vp, vp, i64, vp, vp, C.c_int, i64, vp, vp], C.c_int),
    "snvrag_posfeat": ([i64, i64, vp, C.POINTER(PosfeatW), vp, vp], C.c_int),
    "snvrag_af_gate": ([C.c_int, i64, i64, vp, vp, C.POINTER(AfGateW), vp, vp], C.c_int),
    "snvrag_rag_weighted_concat": ([C.c_int, i64, i64, vp, vp, vp, i64, vp, vp], C.c_int),
    "snvrag_hap_head_out": ([C.c_int, i64, i64, vp, i64, vp, vp, vp, vp, vp], C.c_int),
    "snvrag_gt_head": ([i64, vp, vp, vp, vp, vp, i64, C.POINTER(GtW), vp, vp], C.c_int),
    "snvrag_knn_lut_bytes": ([i64, i32, C.c_int], sz),
    "snvrag_knn_lut": ([i64, i64, i64, vp, vp, vp, i64, vp, vp, i32, i32, C.c_int, C.c_int, C.c_int,
                        C.c_int, vp, vp, vp, vp], C.c_int),
    "snvrag_knn_lut_panel": ([i64, i64, i64, vp, vp, vp, vp, i64, vp, vp, i32, i32, C.c_int, C.c_int, C.c_int,
                              C.c_int, vp, vp, vp, vp], C.c_int),
    "snvrag_knn_scan_parts": ([i64, i32], C.c_int),
    "snvrag_knn_scan": ([vp, i64, i64, i32, vp, i32, C.c_int, C.c_int, i64, vp, i32, vp, vp], C.c_int),
    "snvrag_knn_threshold": ([vp, i32, C.c_int, vp, vp], C.c_int),
    "snvrag_topk_merge_ws_bytes": ([i32, i32, C.c_int], sz),
    "snvrag_topk_merge": ([vp, i32, i32, C.c_int, vp, vp, sz, vp], C.c_int),
    "snvrag_knn_decode": ([vp, i32, C.c_int, vp, vp, vp, vp, vp], C.c_int),
    "snvrag_knn_emb_splits": ([i64, i64, C.c_int], C.c_int),
    "snvrag_knn_emb_ws_bytes": ([i64, C.c_int, C.c_int], sz),
    "snvrag_knn_emb_packed_bytes": ([i64, i64], sz),
    "snvrag_knn_emb_pack": ([vp, i64, i64, vp, vp], C.c_int),
    "snvrag_knn_emb_scan": ([vp, i64, i64, vp, C.c_int, C.c_int, vp, vp], C.c_int),
    "snvrag_knn_emb_finish": ([vp, C.c_int, C.c_int, i64, vp, vp, vp, vp], C.c_int),
    "snvrag_rag_mean": ([C.c_int, i64, i64, i64, C.c_int, vp, vp, i64, i32, vp, vp, vp, C.c_int, C.c_int,
                         C.c_int, C.c_int, C.c_int, vp, vp], C.c_int),
    "snvrag_panel_synth": ([vp, i64, i64, i32, vp, C.c_uint64, vp], C.c_int),
    "snvrag_hamming_lists": ([i64, i64, i32, C.c_int, vp, vp, vp, vp], C.c_int),
    "snvrag_hamming_list_count": ([], i32),
    "snvrag_panel_synth_rows": ([vp, i64, i64, i64, i32, vp, C.c_uint64, vp], C.c_int),
    "snvrag_neighbor_counts": ([i64, C.c_int, vp, vp, i64, i64, i64, vp, i64, vp], C.c_int),
    "snvrag_rag_mean_counts": ([C.c_int, i64, i64, i64, C.c_int, vp, vp, i64, i32, vp, vp, vp, C.c_int, C.c_int,
                                C.c_int, C.c_int, C.c_int, vp, vp], C.c_int),
    "snvrag_encoder_ws_bytes": ([C.c_int, i64, i64, C.c_int, C.c_int], sz),
    "snvrag_encoder_forward": ([C.c_int, i64, i64, C.c_int, C.c_int, C.c_int, C.POINTER(LayerW), vp, vp, sz, vp],
                               C.c_int),
    "snvrag_proj_pack_bytes": ([C.c_int, C.c_int], C.c_size_t),
    "snvrag_proj_pack": ([C.c_int, C.c_int, vp, vp, vp], C.c_int),
    "snvrag_proj_forward": ([i64, C.c_int, C.c_int, vp, vp, vp, vp, vp], C.c_int),
    "snvrag_tail_pack_bytes": ([C.c_int], C.c_size_t),
    "snvrag_tail_pack": ([C.c_int, vp, vp, vp, vp, vp], C.c_int),
    "snvrag_tail_forward": ([i64, C.c_int, vp, vp, vp, vp, vp, vp, vp, f32, vp], C.c_int),
    "snvrag_tail_ffn_forward": ([i64, C.c_int, vp, vp, vp, vp, f32, vp], C.c_int),
    "snvrag_tail_stamps": ([vp], C.c_int),
    "snvrag_attention_train_fwd": ([i64, i64, C.c_int, C.c_int, vp, i64, vp, i64, vp, f32, f32, C.c_uint64, vp],
                                   C.c_int),
    "snvrag_attention_bwd": ([i64, i64, C.c_int, C.c_int, vp, i64, vp, i64, vp, i64, vp, vp, vp, i64, f32, f32,
                              C.c_uint64, vp], C.c_int),
    "snvrag_focal_loss": ([i64, C.c_int, vp, vp, vp, f32, f32, vp, vp, vp], C.c_int),
    "snvrag_sqnorm": ([i64, vp, vp, vp], C.c_int),
    "snvrag_sqnorm_ws_bytes": ([], sz),
    "snvrag_sqnorm_ws": ([i64, vp, vp, vp, sz, vp], C.c_int),
    "snvrag_adam_step": ([i64, vp, vp, vp, vp, vp, vp, C.POINTER(AdamS), vp], C.c_int),
    "snvrag_confusion": ([i64, C.c_int, vp, vp, vp, vp, vp, vp], C.c_int),
    "snvrag_infer_post": ([i64, vp, vp, vp, vp, vp, vp], C.c_int),
    "snvrag_mlp_pack_bytes": ([C.c_int], sz),
    "snvrag_mlp_pack": ([C.c_int, vp, vp, vp, vp], C.c_int),
    "snvrag_mlp_forward": ([i64, C.c_int, C.c_int, vp, vp, vp, vp, vp, i64, f32, vp, vp], C.c_int),
    "snvrag_mlp_afgate_forward": ([i64, C.c_int, vp, vp, vp, f32, vp, vp, vp, vp], C.c_int),
    "snvrag_sgemm_cat_forward": ([i64, C.c_int, C.c_int, vp, vp, vp, i64, vp, vp, vp, vp], C.c_int),
    "snvrag_sgemm_pack_bytes": ([C.c_int, C.c_int], sz),
    "snvrag_sgemm_pack": ([C.c_int, C.c_int, vp, vp, vp], C.c_int),
    "snvrag_derive": ([vp, C.c_int, i64, vp], C.c_int),
    "snvrag_gemm256_pack_bytes": ([C.c_int, C.c_int], sz),
    "snvrag_gemm256_pack": ([C.c_int, C.c_int, vp, i64, vp, vp], C.c_int),
    "snvrag_gemm256_forward": ([i64, C.c_int, C.c_int, vp, i64, vp, vp, vp, i64, vp, i64, vp], C.c_int),
    "snvrag_gemm256_ln_forward": ([i64, C.c_int, C.c_int, vp, i64, vp, vp, vp, vp, C.c_float, vp, i64, C.c_float,
                                   vp, i64, vp, i64, vp], C.c_int),
    "snvrag_head2_fwd": ([i64, C.c_int, vp, vp, vp, vp, vp], C.c_int),
    "snvrag_head2_ws_bytes": ([i64, C.c_int], sz),
    "snvrag_tokgrad_ws_bytes": ([i64, C.c_int, C.c_int], sz),
    "snvrag_tokgrad": ([i64, C.c_int, C.c_int, C.c_int, vp, vp, vp, vp, sz, vp], C.c_int),
    "snvrag_head2_bwd": ([i64, C.c_int, vp, vp, vp, vp, vp, C.c_int, vp, sz, vp], C.c_int),
    "snvrag_sgemm_forward": ([i64, C.c_int, C.c_int, C.c_int, C.c_int, f32, vp, vp, vp, vp, vp, i64, f32, vp, vp, vp,
                              vp], C.c_int),
    "snvrag_ln_fwd_train": ([i64, C.c_int, vp, vp, vp, vp, f32, vp, vp, vp, f32, f32, C.c_uint64, vp], C.c_int),
    "snvrag_nbr_mean_drop_fwd": ([i64, C.c_int, i64, C.c_int, C.c_int, i64, C.c_int, vp, vp, vp, vp, vp, f32,
                                  C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp], C.c_int),
    "snvrag_nbr_mean_drop_bwd": ([i64, C.c_int, i64, C.c_int, C.c_int, i64, C.c_int, vp, vp, vp, vp, vp, f32,
                                  C.c_uint64, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, vp, vp], C.c_int),
    "snvrag_ln_fwd_train_act": ([i64, C.c_int, vp, vp, vp, vp, f32, vp, vp, vp, f32, f32, C.c_uint64, f32, f32, vp],
                                C.c_int),
    "snvrag_ln_bwd_act": ([i64, C.c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp, C.c_int, f32, f32, C.c_uint64, f32, f32,
                           vp, sz, vp], C.c_int),
    "snvrag_ln_bwd_ws_bytes": ([i64, C.c_int], sz),
    "snvrag_ln_bwd": ([i64, C.c_int, vp, vp, vp, vp, vp, vp, vp, vp, C.c_int, f32, f32, C.c_uint64, vp, sz, vp],
                      C.c_int),
    "snvrag_colsum_ws_bytes": ([i64, C.c_int], sz),
    "snvrag_colsum_bf16": ([i64, C.c_int, vp, vp, vp, sz, vp], C.c_int),
    "snvrag_dw_splits": ([i64, i64, i64], C.c_int),
    "snvrag_linear_dw": ([i64, i64, i64, vp, i64, vp, i64, vp, vp, C.c_int, vp], C.c_int),
    "snvrag_linear_dw_parts": ([i64, i64, i64, vp, i64, vp, i64, C.c_int, C.POINTER(vp), C.POINTER(vp), C.c_int, vp],
                               C.c_int),
    "snvrag_evlog_enable": ([C.c_int], C.c_int),
    "snvrag_evlog_pause": ([C.c_int], C.c_int),
    "snvrag_evlog_reset": ([], C.c_int),
    "snvrag_evlog_read": ([vp, vp, vp, C.c_int], C.c_int),
    "snvrag_selftest_mfma": ([vp], C.c_int),
}

EXPORTED = tuple(_SIGS)
_lib: Optional[C.CDLL] = None


class NativeUnavailable(RuntimeError):
    pass


def load(path: Path | str | None = None) -> C.CDLL:
    """Load (once) and type the library.  Raises NativeUnavailable if it is not built."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = Path(path) if path is not None else LIB_PATH
    if not p.exists():
        raise NativeUnavailable(f"{p} not found — build it with `make -C {PKG_DIR}` "
                                "(there is no CPU fallback for the hot path)")
    lib = C.CDLL(str(p))
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes, fn.restype = args, res
    if lib.snvrag_abi_version() != ABI_VERSION:
        raise NativeUnavailable(f"ABI mismatch: lib {lib.snvrag_abi_version()} != {ABI_VERSION}")
    if path is None:
        _lib = lib
    return lib


def lib() -> C.CDLL:
    return load()


def check(rc: int, what: str = "snvrag") -> None:
    if rc != 0:
        msg = lib().snvrag_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


def require_gpu(*tensors: torch.Tensor) -> None:
    if not torch.cuda.is_available():
        raise NativeUnavailable("no HIP device: the SNV-RAG hot path runs only on the GPU (no CPU fallback)")
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise ValueError("expected device tensors (got a CPU tensor)")


def stream_ptr(stream: Optional[torch.cuda.Stream] = None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else int(t.data_ptr())


def dtype_code(dt: torch.dtype) -> int:
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    raise ValueError(f"unsupported dtype {dt}")
