"""torch.autograd Functions over the libsnvrag training kernels.

The training graph (``src/train_forward.py``) is ordinary autograd; its heavy nodes
are these Functions, whose forward and backward run the HIP kernels:

  hip_linear      Linear layers on the MFMA GEMMs (bf16 in, f32 accumulate):
                  forward  y = x W^T + b             (stream GEMM at K = 384, wide-row GEMM for
                                                      the large-K -> 384 ones, else snvrag_linear)
                  backward dx = dy W                 (the same GEMMs on W^T)
                           dW = dy^T x, db = sum dy  (snvrag_linear_dw: split-M MFMA kernel on
                                                      LDS-transposed tiles, f32 result; shapes
                                                      that are not multiples of 128 (the AF MLP's
                                                      64 inputs) on torch.mm with an f32 result)
  hip_attention   unmasked softmax attention: flash forward that keeps the row
                  log-sum-exp, FlashAttention-2 style dq / dkv backward kernels.
  focal_loss      FocalLoss(reduction='sum') over masked rows, forward and derivative
                  fused in one kernel.
  rag_mean_train  K-mean of the retrieved neighbours' complete-token embeddings
                  (embedding_rag_dataset.py:404-438 re-encode WITH grad + bert.py:176-179
                  mean): values from the rag_mean kernel; gradients into the token
                  table (rows tok0/tok1/<sos>/<eos>, <pad> excluded as nn.Embedding's
                  padding_idx) and into the panel AF embedding.

Master parameters stay f32 ``nn.Parameter``s; their bf16 compute copies are cached per
parameter version (the fused Adam kernel bumps the version in place).
"""

from __future__ import annotations

import contextlib
import os
import weakref
from typing import Dict, Optional, Tuple

import torch

from . import kernels as K

_TRAIN_DT = [torch.bfloat16]              # compute dtype of the training graph


def train_dtype() -> torch.dtype:
    return _TRAIN_DT[0]


def set_train_precision(dtype: torch.dtype) -> None:
    """Compute dtype of the training graph: torch.bfloat16 (the product path: bf16 MFMA kernels,
    f32 accumulation and master weights) or torch.float32 — the gradient-parity mode, whose
    parameter gradients are held to 1e-3 of the reference's own autograd
    (tests/test_gpu_train.py): every Linear on the exact-f32 row-panel MFMA GEMM (forward and
    dX; f32 dW), LayerNorm and attention as f32 torch ops."""
    if dtype not in (torch.float32, torch.bfloat16):
        raise ValueError("training precision must be float32 or bfloat16")
    _TRAIN_DT[0] = dtype


_BF16: Dict[tuple, list] = {}
_MIRROR: Dict[int, tuple] = {}              # id(param) -> (weakref(param), flat-buffer bf16 view)
_EPOCH = [0]                                # bumped after every optimizer step


def _base_key(p: torch.Tensor):
    base = p._base if p._base is not None else p
    return base, (id(base), p.storage_offset(), tuple(p.shape), tuple(p.stride()))


def bf16_of(p: torch.Tensor, transposed: bool = False) -> torch.Tensor:
    """bf16 copy (or transposed copy) of a master parameter (or a view of one).  Entries are
    tied to the live base tensor (weakref identity, so a freed parameter's address reused by
    another can never hit) and to (its version, the optimizer epoch).  Parameters held in a
    FlatParams buffer read the optimizer's bf16 mirror directly."""
    if not transposed and p._base is None:
        mv = _MIRROR.get(id(p))
        if mv is not None and mv[0]() is p:
            return mv[1]
    if p.dtype != torch.float32 or not p.is_cuda or p.dim() != 2:
        base, key = _base_key(p)
        ent = _BF16.get(key)
        ver = (base._version, _EPOCH[0])
        if ent is None or ent[0]() is not base or ent[1] != ver:
            ent = [weakref.ref(base), ver, p.detach().to(torch.bfloat16).contiguous(), None]
            _BF16[key] = ent
        if not transposed:
            return ent[2]
        if ent[3] is None:
            ent[3] = ent[2].t().contiguous()
        return ent[3]
    src = p.detach().t() if transposed else p.detach()
    return _derived(("bf16", transposed), [p], lambda: _plain_job(K.DERIVE_BF16, [src]))


def clear_weight_cache() -> None:
    _BF16.clear()
    _DER.clear()
    _DER_TABLE[0] = None


def weights_updated() -> None:
    """Called after a parameter update done outside torch's version tracking (HIP kernels):
    every derived weight tensor is refreshed from the new master weights in one launch.

    Every call also counts as a weight change for the train-mode retrieval's panel snapshot
    (``embedding_rag_dataset._weights_token``): after it the window's stale-snapshot search takes
    the exact LUT form even if the values did not change (an lr = 0 step, ``sync_mirror``) — the
    same neighbours, a slower LUT.  On a sharded panel that decision selects collectives
    (``any_rank``), so every rank must make the same calls in the same order: the trainer calls it
    once per optimizer step and once per ``load`` / ``sync_mirror``, on every rank alike."""
    _EPOCH[0] += 1
    _BF16.clear()
    _refresh_derived()


# Derived weight tensors (stream-GEMM packs, transposed / concatenated bf16 copies, bias tables)
# of f32 master parameters.  An entry is built once (buffers allocated, its jobs run at once)
# and then REFRESHED IN PLACE: after every optimizer step all live entries are recomputed by
# one snvrag_derive launch over a cached device job table (round 3 rebuilt each of them at its
# first use in the step with fresh allocations, cats, transposes and one pack kernel apiece:
# ~150 cat / ~70 pack / ~50 copy launches per training step).  A torch-side in-place update
# (version bump) refreshes the entry at its next use; a moved or freed source drops it.
class _Derived:
    __slots__ = ("refs", "ptrs", "vers", "jobs", "out")


_DER: Dict[tuple, _Derived] = {}
_DER_TABLE = [None]                         # (device job table, njobs, pieces) over all of _DER


def _parts_state(parts):
    bases = [_base_key(t)[0] for t in parts]
    return bases, tuple(b.data_ptr() for b in bases), tuple(b._version for b in bases)


def _plain_job(kind, srcs, shape=None):
    """(out, [job]): the f32 / bf16 row-major copy of the row-stacked f32 views ``srcs``."""
    rows = sum(t.shape[0] for t in srcs)
    cols = srcs[0].shape[1] if srcs[0].dim() == 2 else 1
    dt = torch.float32 if kind == K.DERIVE_F32 else torch.bfloat16
    out = torch.empty(shape or ((rows, cols) if srcs[0].dim() == 2 else (rows,)), device=srcs[0].device, dtype=dt)
    return out, [K.derive_job(kind, [t.detach() for t in srcs], out)]


def _derived(tag: tuple, parts, make):
    """The derived tensor(s) ``make() -> (out, jobs)`` of the f32 parameters (or views) ``parts``,
    current for their present values."""
    keys = [_base_key(t)[1] for t in parts]
    key = tag + tuple(keys)
    bases, ptrs, vers = _parts_state(parts)
    ent = _DER.get(key)
    if ent is None or ent.ptrs != ptrs or any(r() is not b for r, b in zip(ent.refs, bases)):
        ent = _Derived()
        ent.out, ent.jobs = make()
        ent.refs, ent.ptrs, ent.vers = [weakref.ref(b) for b in bases], ptrs, vers
        _DER[key] = ent
        _DER_TABLE[0] = None
        K.derive(K.derive_table(ent.jobs, bases[0].device))
    elif ent.vers != vers:
        K.derive(K.derive_table(ent.jobs, bases[0].device))
        ent.vers = vers
    return ent.out


def _refresh_derived() -> None:
    dead, live = [], []                     # live: strong references to the sources until the launch
    for key, ent in _DER.items():
        bases = [r() for r in ent.refs]
        if any(b is None for b in bases) or tuple(b.data_ptr() for b in bases) != ent.ptrs:
            dead.append(key)
        else:
            ent.vers = tuple(b._version for b in bases)
            live.append(bases)
    for key in dead:
        del _DER[key]
        _DER_TABLE[0] = None
    if not _DER:
        return
    if _DER_TABLE[0] is None:
        jobs = [j for ent in _DER.values() for j in ent.jobs]
        _DER_TABLE[0] = K.derive_table(jobs, live[0][0].device)
    K.derive(_DER_TABLE[0])


def register_mirror(p: torch.Tensor, view: torch.Tensor) -> None:
    _MIRROR[id(p)] = (weakref.ref(p), view)


class _TinyVocabEmbedding(torch.autograd.Function):
    """W[tok] (F.embedding with padding_idx) for a vocabulary of a few rows: the weight gradient
    is one one-hot GEMM (onehot(tok)^T grad, reads grad once) instead of embedding_dense_backward's
    sort + segment scatter, which took ~6 ms per call on the 4e5 re-encoded neighbour tokens
    (embedding_rag_dataset.py:404-417) into the 10-row token table."""

    @staticmethod
    def forward(ctx, tok, W, padding_idx):
        ctx.save_for_backward(tok)
        ctx.V, ctx.padding_idx, ctx.wdtype = W.shape[0], padding_idx, W.dtype
        return torch.nn.functional.embedding(tok, W, padding_idx=padding_idx)

    @staticmethod
    def backward(ctx, g):
        (tok,) = ctx.saved_tensors
        D = g.shape[-1]
        if ctx.V <= 16 and D % 2 == 0 and g.is_cuda:
            # one pass over g, per-block partials + fixed-order sum (csrc/train.hip tokgrad)
            return None, K.tokgrad(tok, g, ctx.V, ctx.padding_idx).to(ctx.wdtype), None
        oh = torch.nn.functional.one_hot(tok.reshape(-1), ctx.V).to(torch.float32)
        gW = oh.t() @ g.reshape(-1, D).float()
        if ctx.padding_idx is not None:
            gW[ctx.padding_idx] = 0
        return None, gW.to(ctx.wdtype), None


def tiny_embedding(tok: torch.Tensor, W: torch.Tensor, padding_idx: Optional[int] = 0) -> torch.Tensor:
    """F.embedding(tok, W, padding_idx) with the one-hot-GEMM weight gradient (small vocabularies)."""
    if not (W.requires_grad and torch.is_grad_enabled()):
        return torch.nn.functional.embedding(tok, W, padding_idx=padding_idx)
    return _TinyVocabEmbedding.apply(tok, W, padding_idx)


def _sg_stream(ws, bs, n_out: int, extra=()):
    """(packed weight stream, f32 vector table) of the stream GEMM (csrc/sgemm.hip) for the
    weights ``ws`` (f32 [n_i, K] parameters or views, concatenated along the outputs) and biases
    ``bs`` (+ ``extra`` f32 columns appended to the table: the rank-2 linear's W[:, D], W[:, D+1])."""
    parts = list(ws) + [b for b in bs if b is not None] + list(extra)

    def make():
        Kd = ws[0].shape[1]
        packed = torch.empty(int(K.N.lib().snvrag_sgemm_pack_bytes(Kd, n_out)), device=ws[0].device,
                             dtype=torch.uint8)
        jobs = [K.derive_job(K.DERIVE_SGPACK, [w.detach() for w in ws], packed)]
        if bs[0] is None and not extra:
            vec = torch.zeros(n_out, device=ws[0].device, dtype=torch.float32)
        else:
            vec, vj = _plain_job(K.DERIVE_F32, [t.detach().reshape(-1) for t in bs if t is not None] +
                                 [t.detach() for t in extra])
            jobs += vj
        return (packed, vec), jobs
    return _derived(("sg", len(extra)), parts, make)


def _cat_bf16(ws, transposed: bool = False) -> torch.Tensor:
    """bf16 cat(ws, 0) (or its transpose) of f32 weights, refreshed with the derived tensors."""
    def make():
        rows, cols = sum(w.shape[0] for w in ws), ws[0].shape[1]
        if not transposed:
            return _plain_job(K.DERIVE_BF16, list(ws))
        out = torch.empty(cols, rows, device=ws[0].device, dtype=torch.bfloat16)
        jobs, off = [], 0
        for w in ws:                                # column block of the transposed output
            jobs.append(K.derive_job(K.DERIVE_BF16, [w.detach().t()], out.view(-1)[off:], dst_ld=rows))
            off += w.shape[0]
        return out, jobs
    return _derived(("catT" if transposed else "cat",), list(ws), make)


def _cat_f32(bs) -> torch.Tensor:
    return _derived(("bcat",), list(bs), lambda: _plain_job(K.DERIVE_F32, [t.detach().reshape(-1) for t in bs]))


def _sg_stream_t(w: torch.Tensor, n_out: int):
    """Packed stream of W^T (the dX = dY W GEMM of a single Linear with out_features = 384)."""
    def make():
        wt = w.detach().t()
        packed = torch.empty(int(K.N.lib().snvrag_sgemm_pack_bytes(wt.shape[1], wt.shape[0])), device=w.device,
                             dtype=torch.uint8)
        return (packed, torch.zeros(n_out, device=w.device, dtype=torch.float32)), \
            [K.derive_job(K.DERIVE_SGPACK, [wt], packed)]
    return _derived(("sgT",), [w], make)


def _g2_stream(ws, bs):
    """(packed stream, f32 bias or None) of the wide-row GEMM (csrc/gemm256.hip) for the weights
    ``ws`` concatenated along the outputs (FeedForward's w_2: one [384, 1536] weight)."""
    parts = list(ws) + [b for b in bs if b is not None]

    def make():
        n_out, Kd = sum(w.shape[0] for w in ws), ws[0].shape[1]
        packed = torch.empty(int(K.N.lib().snvrag_gemm256_pack_bytes(n_out, Kd)), device=ws[0].device,
                             dtype=torch.uint8)
        jobs = [K.derive_job(K.DERIVE_G2PACK, [w.detach() for w in ws], packed)]
        if bs[0] is None:
            return (packed, None), jobs
        vec, vj = _plain_job(K.DERIVE_F32, [t.detach().reshape(-1) for t in bs])
        return (packed, vec), jobs + vj
    return _derived(("g2",), parts, make)


def _g2_stream_t(ws):
    """Packed stream of [W_1; ..; W_n]^T for the wide-row GEMM (the dX = dY [W_1; ..; W_n] GEMM
    onto 384 inputs): the pack is K-major, so the pack of the column blocks W_i^T is the
    concatenation of their packs — one derive job per weight."""
    def make():
        n_in = ws[0].shape[1]
        total = int(K.N.lib().snvrag_gemm256_pack_bytes(n_in, sum(w.shape[0] for w in ws)))
        packed = torch.empty(total, device=ws[0].device, dtype=torch.uint8)
        jobs, off = [], 0
        for w in ws:
            nb = int(K.N.lib().snvrag_gemm256_pack_bytes(n_in, w.shape[0]))
            jobs.append(K.derive_job(K.DERIVE_G2PACK, [w.detach().t()], packed[off:off + nb]))
            off += nb
        return packed, jobs
    return _derived(("g2T",), list(ws), make)


def _g2_ok(k_in: int, n_out: int, parts=()) -> bool:
    """The wide-row GEMM takes the large-K projections onto 384 features: FeedForward's w_2
    forward (K = 4D) and the dX GEMMs of q/k/v (K = 3D) and w_1 (K = 4D).  62 / 49 us at
    M = 49 440, K = 1536 / 1152, vs hipBLASLt's 68-78 / 54-58 and the row panel's 78 / 60
    (tools/gemm256_micro.py)."""
    return (n_out == 384 and k_in >= 1024 and k_in % 64 == 0 and all(t % 64 == 0 for t in parts)
            and not _BLAS_LARGE_K[0])


def _sg_ok(x2: torch.Tensor, n_out: int) -> bool:
    """The stream GEMM takes the K = 384, no-activation projections (QKV, FFN w_1, fusion /
    head Linear layers): 850-900 TFLOP/s vs the row panel's ~550 at the training shapes."""
    return (x2.shape[-1] == 384 and n_out % 64 == 0 and x2.shape[0] * n_out * 2 < (1 << 31)
            and not os.environ.get("SNVRAG_TRAIN_NO_SG"))


_MM_F32_OUT = None


def _mm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a @ b (bf16) with an f32 result written by the GEMM itself (aten::mm.dtype on ROCm:
    f32 accumulate, f32 store) — the weight gradient keeps its f32 accumulation instead of being
    rounded to bf16 and widened again by a separate conversion kernel.  Where the dtype overload
    is unavailable it falls back to the bf16-output GEMM + widening and says so (once): the
    weight gradients are then bf16-rounded."""
    global _MM_F32_OUT
    if _MM_F32_OUT is None:
        try:
            torch.mm(a[:8, :8], b[:8, :8], out_dtype=torch.float32)
            _MM_F32_OUT = True
        except (RuntimeError, TypeError, NotImplementedError) as e:
            _MM_F32_OUT = False
            import warnings
            warnings.warn(f"torch.mm(..., out_dtype=float32) unavailable ({e!r}): weight gradients fall back "
                          "to a bf16-output GEMM (bf16-rounded dW)", RuntimeWarning, stacklevel=2)
    if _MM_F32_OUT:
        return torch.mm(a, b, out_dtype=torch.float32)
    return torch.mm(a, b).float()


def _wgrad(g2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    """f32 dW = g2^T x2 for a small weight (N x K <= 2^18) over many rows M: the library GEMM runs
    such an output on a handful of workgroups looping the whole M (47-107 us per call at M = 24 720 /
    49 440, ~0.8 ms per training step over the AF MLPs, the rag-fusion gate / encoder and the
    genotype head); here M is cut into 64 row chunks — one batched GEMM over the chunks, then the
    fixed-order sum of the 64 partial products (plus the < 64 leftover rows)."""
    M, N = g2.shape
    Kd = x2.shape[1]
    if M < 8192 or N * Kd > (1 << 18):
        return _mm_f32(g2.t(), x2) if g2.dtype == torch.bfloat16 else g2.float().t() @ x2.float()
    g2, x2 = g2.float().contiguous(), x2.float().contiguous()
    C = 64
    Mc = M // C
    main = C * Mc
    out = torch.bmm(g2[:main].reshape(C, Mc, N).transpose(1, 2), x2[:main].reshape(C, Mc, Kd)).sum(0)
    if main < M:
        out += g2[main:].t() @ x2[main:]
    return out


class _SmallLinear(torch.autograd.Function):
    """nn.Linear in f32 for the small per-site MLPs (rag fusion's gate / joint encoder,
    fusion.py:82-128; the genotype head, foundation_model.py:64-80): torch's forward and dX,
    the weight gradient by :func:`_wgrad`."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_b = b is not None
        return torch.nn.functional.linear(x, w, b)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        N, Kd = w.shape
        g2 = g.reshape(-1, N)
        gx = (g @ w.to(g.dtype)).to(x.dtype) if ctx.needs_input_grad[0] else None
        gw = _wgrad(g2, x.reshape(-1, Kd)).to(w.dtype) if ctx.needs_input_grad[1] else None
        gb = g2.float().sum(0).to(w.dtype) if ctx.has_b and ctx.needs_input_grad[2] else None
        return gx, gw, gb


def small_linear(x: torch.Tensor, lin) -> torch.Tensor:
    """``lin(x)`` for an nn.Linear whose weight gradient is a small output over many rows."""
    if not torch.is_grad_enabled() or not x.is_cuda:
        return torch.nn.functional.linear(x, lin.weight, lin.bias)
    return _SmallLinear.apply(x, lin.weight, lin.bias)


_DIRECT_GRADS = False
_BLAS_LARGE_K = [False]                     # A/B only: the large-K -> 384 GEMMs on hipBLASLt


def set_blas_dx(enabled: bool) -> bool:
    """A/B switch (tools/train_only.py BLAS_DX=1): the large-K -> 384 GEMMs of training (w_2
    forward, the q/k/v and w_1 dX) on hipBLASLt instead of the wide-row kernel (the default).
    Returns the previous setting."""
    prev = _BLAS_LARGE_K[0]
    _BLAS_LARGE_K[0] = bool(enabled)
    return prev


@contextlib.contextmanager
def direct_weight_grads(enabled: bool = True):
    """Inside this context (the trainer's ``loss.backward()``), Linear backward accumulates dW
    and db straight into the parameters' f32 ``.grad`` (the flat gradient buffer of
    ``FlatParams``) with the dW kernel, instead of returning fresh tensors that autograd then
    adds in with one kernel per parameter (and zero-fills before: ~300 small launches per
    step).  Autograd still runs each such parameter's AccumulateGrad node once per backward,
    after the LAST use of the parameter has run its backward (with an undefined gradient, so
    nothing is added), and its post-accumulate hooks fire there — exactly once per parameter
    and step, which is what ``GradBucketer`` keys its bucket launches on.  Outside the context
    (e.g. ``torch.autograd.grad``), gradients are returned as usual."""
    global _DIRECT_GRADS
    prev = _DIRECT_GRADS
    _DIRECT_GRADS = enabled
    try:
        yield
    finally:
        _DIRECT_GRADS = prev


def _grad_buffer(p) -> Optional[torch.Tensor]:
    g = p.grad if (p is not None and p.is_leaf and p.requires_grad) else None
    return g if (g is not None and g.dtype == torch.float32 and g.is_contiguous()) else None


class GradHandoff:
    """A gradient handed from one backward to another instead of through autograd's accumulation.

    In a transformer block the stream tensor x feeds both the next GEMM (the q/k/v projection, or
    FeedForward's w_1) and the add+LayerNorm that closes the sublayer (sublayer.py:15-16:
    norm(x + sublayer(x))).  Autograd would receive x's gradient twice and add the two [M, D]
    tensors with one more elementwise kernel per sublayer (24 per step at d384/L12).  With a
    handoff, the add+LayerNorm backward (which runs first: its other operand depends on the GEMM)
    deposits its dx here and returns no gradient for x, and the GEMM's dX backward adds it in its
    epilogue (the row-panel GEMM's residual operand: one f32 accumulate + one bf16 rounding)."""
    __slots__ = ("g",)

    def __init__(self):
        self.g = None

    def take(self) -> Optional[torch.Tensor]:
        g, self.g = self.g, None
        return g


class _HipLinear(torch.autograd.Function):
    """y = x [W_1; ..; W_n]^T + [b_1; ..; b_n]: one GEMM over weights concatenated along the
    output dim (the q/k/v Linear layers of multi_head_attention.py:44 as one N = 3D GEMM)."""

    @staticmethod
    def forward(ctx, x, n, handoff, *wb):
        ws, bs = wb[:n], wb[n:]
        ctx.handoff = handoff
        Kd = x.shape[-1]
        if train_dtype() == torch.float32:
            return _HipLinear._forward_f32(ctx, x, n, ws, bs)
        x2 = x.reshape(-1, Kd)
        if x2.dtype != torch.bfloat16:
            x2 = x2.to(torch.bfloat16)
        x2 = x2.contiguous()
        has_b = bs[0] is not None
        n_out = sum(t.shape[0] for t in ws)
        if _sg_ok(x2, n_out):
            wsp, vec = _sg_stream(ws, bs, n_out)
            y = K.sgemm(x2, wsp, n_out, vec)
        elif _g2_ok(Kd, n_out, [t.shape[0] for t in ws]):
            # FeedForward's w_2 (K = 4D -> D) on the wide-row GEMM, f32 bias in its epilogue
            wsp, vec = _g2_stream(ws, bs)
            y = K.gemm256(x2, wsp, n_out, bias=vec)
        elif _BLAS_LARGE_K[0] and n == 1 and Kd >= 1024 and n_out == 384:
            w = bf16_of(ws[0])                      # A/B: hipBLASLt (bias taken in bf16)
            y = torch.addmm(bf16_of(bs[0]), x2, w.t()) if has_b else torch.mm(x2, w.t())
        else:
            w = bf16_of(ws[0]) if n == 1 else _cat_bf16(ws)
            b = (bs[0].detach() if n == 1 else _cat_f32(bs)) if has_b else None
            y = K.linear(x2, w, b)
        ctx.save_for_backward(x2, *ws)
        ctx.n, ctx.has_bias = n, has_b
        ctx.in_shape, ctx.in_dtype = x.shape, x.dtype
        ctx.params = (ws, bs)                       # leaves: for the direct .grad accumulation
        return y.reshape(*x.shape[:-1], n_out)

    @staticmethod
    def _forward_f32(ctx, x, n, ws, bs):
        """Parity mode: y = x W^T + b on the exact-f32 row-panel GEMM (v_mfma_f32_16x16x4f32)."""
        x2 = x.reshape(-1, x.shape[-1]).float().contiguous()
        w = torch.cat([t.detach().float() for t in ws], 0).contiguous()
        has_b = bs[0] is not None
        b = torch.cat([t.detach().float().reshape(-1) for t in bs]).contiguous() if has_b else None
        y = K.linear(x2, w, b)
        ctx.save_for_backward(x2, *ws)
        ctx.n, ctx.has_bias, ctx.f32 = n, has_b, True
        ctx.in_shape, ctx.in_dtype = x.shape, x.dtype
        return y.reshape(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, gy):
        if getattr(ctx, "f32", False):
            return _HipLinear._backward_f32(ctx, gy)
        x2, *ws = ctx.saved_tensors
        sizes = [t.shape[0] for t in ws]
        g2 = gy.reshape(-1, sum(sizes))
        if g2.dtype != torch.bfloat16:
            g2 = g2.to(torch.bfloat16)
        g2 = g2.contiguous()
        gx = None
        gws = [None] * ctx.n
        gbs = [None] * ctx.n
        res = ctx.handoff.take() if ctx.handoff is not None else None
        if ctx.needs_input_grad[0]:
            n_in = ctx.in_shape[-1]
            if ctx.n == 1 and _sg_ok(g2, n_in):
                wsp, vec = _sg_stream_t(ws[0], n_in)
                gx = K.sgemm(g2, wsp, n_in, vec)
                if res is not None:
                    gx += res.reshape(gx.shape).to(gx.dtype)
            elif _g2_ok(g2.shape[1], n_in, sizes):
                # the K >= 1024 -> 384 dX GEMMs (q/k/v, FeedForward w_1) on the wide-row GEMM; the
                # handed-off gradient enters its epilogue (one f32 add, one rounding) into a fresh
                # output (the handed-off tensor may also be another node's returned gradient)
                wsp = _g2_stream_t(ws)
                if res is None:
                    gx = K.gemm256(g2, wsp, n_in)
                else:
                    r2 = res.reshape(-1, n_in).to(torch.bfloat16)
                    if r2.stride(1) != 1 or r2.stride(0) % 8 or r2.data_ptr() % 16:
                        # a fresh, 16-byte aligned copy (contiguous() returns a contiguous but
                        # misaligned view unchanged, which the C side would reject)
                        r2 = r2.clone(memory_format=torch.contiguous_format)
                    gx = K.gemm256(g2, wsp, n_in, resid=r2)
            elif _BLAS_LARGE_K[0] and g2.shape[1] >= 1024 and n_in == 384:
                # A/B: hipBLASLt, the handed-off gradient as addmm's C operand
                wc = bf16_of(ws[0]) if ctx.n == 1 else _cat_bf16(ws)
                gx = torch.mm(g2, wc) if res is None else \
                    torch.addmm(res.reshape(-1, n_in).to(torch.bfloat16), g2, wc)
            else:
                wt = bf16_of(ws[0], transposed=True) if ctx.n == 1 else _cat_bf16(ws, transposed=True)
                gx = K.linear(g2, wt, resid=None if res is None else res.reshape(-1, n_in).to(torch.bfloat16))
            gx = gx.reshape(ctx.in_shape).to(ctx.in_dtype)
        n_all, k_in = g2.shape[1], x2.shape[1]
        dw_ok = n_all % 128 == 0 and k_in % 128 == 0 and all(sz % 128 == 0 for sz in sizes) and \
            not os.environ.get("SNVRAG_TRAIN_BLAS_DW")
        pws, pbs = ctx.params
        if _DIRECT_GRADS and dw_ok and all(_grad_buffer(w) is not None for w in pws) and \
                (not ctx.has_bias or all(_grad_buffer(b) is not None for b in pbs)):
            # accumulate into the flat gradient buffer: one dW launch per weight (its column
            # slice of dy), bias sums fused
            if ctx.n == 1:
                K.linear_dw(g2, x2, dw=pws[0].grad, db=pbs[0].grad if ctx.has_bias else None)
            elif len(set(sizes)) == 1 and ctx.n <= 4:
                K.linear_dw_parts(g2, x2, [w.grad for w in pws], [b.grad for b in pbs] if ctx.has_bias else None)
            else:
                off = 0
                for w, b, sz in zip(pws, pbs, sizes):
                    K.linear_dw(g2[:, off:off + sz], x2, dw=w.grad, db=b.grad if ctx.has_bias else None)
                    off += sz
            return (gx, None, None, *([None] * ctx.n), *([None] * ctx.n))
        if any(ctx.needs_input_grad[3:3 + ctx.n]) and dw_ok:
            # dW (and db) on the split-M MFMA kernel (csrc/dw.hip), f32 accumulation and result
            gw, gb = K.linear_dw(g2, x2, bias=ctx.has_bias)
            gws = list(torch.split(gw, sizes, 0))
            if ctx.has_bias:
                gbs = list(torch.split(gb, sizes, 0))
            return (gx, None, None, *gws, *gbs)
        if any(ctx.needs_input_grad[3:3 + ctx.n]):
            gw = _wgrad(g2, x2)
            gws = list(torch.split(gw, sizes, 0))
        if ctx.has_bias:
            gb = K.colsum(g2) if g2.shape[-1] % 8 == 0 and g2.shape[-1] <= 2048 else g2.float().sum(0)
            gbs = list(torch.split(gb, sizes, 0))
        return (gx, None, None, *gws, *gbs)


def _hip_linear_backward_f32(ctx, gy):
    x2, *ws = ctx.saved_tensors
    sizes = [t.shape[0] for t in ws]
    g2 = gy.reshape(-1, sum(sizes)).float().contiguous()
    gx = None
    if ctx.needs_input_grad[0]:
        wt = torch.cat([t.detach().float() for t in ws], 0).t().contiguous()
        gx = K.linear(g2, wt).reshape(ctx.in_shape).to(ctx.in_dtype)
    res = ctx.handoff.take() if ctx.handoff is not None else None
    if res is not None and gx is not None:
        gx = gx + res.to(gx.dtype)
    gws = list(torch.split(g2.t() @ x2, sizes, 0)) if any(ctx.needs_input_grad[3:3 + ctx.n]) else [None] * ctx.n
    gbs = list(torch.split(g2.sum(0), sizes, 0)) if ctx.has_bias else [None] * ctx.n
    return (gx, None, None, *gws, *gbs)


_HipLinear._backward_f32 = staticmethod(_hip_linear_backward_f32)


def hip_linear(x: torch.Tensor, weight, bias=None, grad_from: Optional[GradHandoff] = None) -> torch.Tensor:
    """nn.Linear on the MFMA kernels; bf16 activations in and out.  ``weight``/``bias`` may be
    lists (layers sharing the input, fused along the output dim).  ``grad_from``: x's other
    gradient, deposited by an add+LayerNorm backward (:class:`GradHandoff`), joins dX."""
    ws = list(weight) if isinstance(weight, (list, tuple)) else [weight]
    bs = list(bias) if isinstance(bias, (list, tuple)) else [bias] * len(ws)
    Kd, Nn = ws[0].shape[1], sum(t.shape[0] for t in ws)
    if Kd % 8 or Nn % 8:
        if train_dtype() == torch.float32:
            assert grad_from is None, "a gradient handoff needs the HIP Linear path"
            b = torch.cat(bs, 0) if bs[0] is not None else None
            return torch.nn.functional.linear(x.float(), torch.cat(ws, 0), b)
        w = torch.cat(ws, 0).to(torch.bfloat16)
        b = torch.cat(bs, 0).to(torch.bfloat16) if bs[0] is not None else None
        assert grad_from is None, "a gradient handoff needs the HIP Linear path"
        return torch.nn.functional.linear(x.to(torch.bfloat16), w, b)
    return _HipLinear.apply(x, len(ws), grad_from, *ws, *bs)


class _Head2(torch.autograd.Function):
    """The hap head's Linear(4D, 2) (foundation_model.py:25-33 net[2]): bf16 activations, f32
    weights and logits (csrc/train.hip head2_*; torch ran F.linear(hh.float(), W): an f32 copy of
    the [M, 4D] activations and N = 2 GEMMs)."""

    @staticmethod
    def forward(ctx, x, w, b):
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        y = K.head2_fwd(x2, w.detach(), b.detach())
        ctx.save_for_backward(x2, w)
        ctx.in_shape, ctx.params = x.shape, (w, b)
        return y.reshape(*x.shape[:-1], 2)

    @staticmethod
    def backward(ctx, gy):
        x2, w = ctx.saved_tensors
        g2 = gy.reshape(-1, 2).float().contiguous()
        pw, pb = ctx.params
        direct = _DIRECT_GRADS and _grad_buffer(pw) is not None and _grad_buffer(pb) is not None
        dx, dw = K.head2_bwd(g2, x2, w.detach(), want_dx=ctx.needs_input_grad[0],
                             dw=pw.grad if direct else None, accumulate=direct)
        gb = g2.sum(0)
        if dx is not None:
            dx = dx.reshape(ctx.in_shape)
        if direct:
            pb.grad.add_(gb)
            return dx, None, None
        return dx, (dw if ctx.needs_input_grad[1] else None), (gb if ctx.needs_input_grad[2] else None)


def head2_linear(x: torch.Tensor, lin) -> torch.Tensor:
    """f32 logits of ``lin`` = nn.Linear(K, 2) on bf16 ``x``; the f32 parity mode keeps
    F.linear on f32 activations."""
    if train_dtype() == torch.float32 or x.dtype != torch.bfloat16 or x.shape[-1] % 8 or \
            tuple(lin.weight.shape) != (2, x.shape[-1]) or lin.bias is None:
        return torch.nn.functional.linear(x.float(), lin.weight, lin.bias)
    return _Head2.apply(x, lin.weight, lin.bias)


class _HipLinearRank2(torch.autograd.Function):
    """z = Linear(cat([x, c1, c2], -1)) = x W[:, :D]^T + b + c1 W[:, D] + c2 W[:, D + 1] (bf16 out)
    with the two extra input columns as per-row rank-1 terms in the stream GEMM's epilogue
    (fusion.py:355-360's cat(emb, pos_feat, af) and foundation_model.py's cat(x, af, af_p)):
    no [M, N] f32 products and adds in torch.  Backward: dX on the stream / row-panel GEMM,
    dW[:, :D] and db on the dW kernel, dW[:, D:] = dz^T [c1 c2] and dc = dz W[:, D:] as two
    skinny products."""

    @staticmethod
    def forward(ctx, x, c1, c2, W, b):
        D = x.shape[-1]
        n_out = W.shape[0]
        x2 = x.reshape(-1, D).to(torch.bfloat16).contiguous()
        M = x2.shape[0]
        r1 = c1.reshape(-1).float().contiguous()
        r2 = c2.reshape(-1).float().contiguous()
        assert r1.numel() == M and r2.numel() == M
        wsp, vec = _sg_stream([W[:, :D]], [b], n_out, extra=(W[:, D], W[:, D + 1]))   # [bias | w_c1 | w_c2]
        z = K.sgemm(x2, wsp, n_out, vec, rank=(r1, r2, M))
        ctx.save_for_backward(x2, r1, r2, W)
        ctx.in_shape, ctx.in_dtype, ctx.D = x.shape, x.dtype, D
        return z.reshape(*x.shape[:-1], n_out)

    @staticmethod
    def backward(ctx, gz):
        x2, r1, r2, W = ctx.saved_tensors
        D, n_out = ctx.D, W.shape[0]
        g2 = gz.reshape(-1, n_out).to(torch.bfloat16).contiguous()
        gx = gc1 = gc2 = gW = gb = None
        wd = W[:, :D]
        if ctx.needs_input_grad[0]:
            if _sg_ok(g2, D):
                wsp, vec = _sg_stream_t(wd, D)
                gx = K.sgemm(g2, wsp, D, vec)
            else:
                gx = K.linear(g2, bf16_of(wd, transposed=True))
            gx = gx.reshape(ctx.in_shape).to(ctx.in_dtype)
        M = g2.shape[0]
        if ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            # dc = dz W[:, D:] on the row-panel GEMM, the two columns padded to 8 outputs
            wc = torch.zeros(8, n_out, device=g2.device, dtype=torch.bfloat16)
            wc[:2] = W[:, D:].detach().t().to(torch.bfloat16)
            gcc = K.linear(g2, wc, out_dtype=torch.float32)            # [M, 8]
            gc1 = gcc[:, 0].reshape(ctx.in_shape[:-1]) if ctx.needs_input_grad[1] else None
            gc2 = gcc[:, 1].reshape(ctx.in_shape[:-1]) if ctx.needs_input_grad[2] else None
        if ctx.needs_input_grad[3] or ctx.needs_input_grad[4]:
            # dW[:, :D] and db, then dW[:, D:] = dz^T [c1 c2] on the same dW kernel with the two row
            # columns padded to one 128-wide operand (skinny library GEMMs over M took ~0.3 ms each)
            gwd, gb = K.linear_dw(g2, x2, bias=True)
            cc = torch.zeros(M, 128, device=g2.device, dtype=torch.bfloat16)
            cc[:, 0] = r1
            cc[:, 1] = r2
            gwc, _ = K.linear_dw(g2, cc)
            gW = torch.cat([gwd, gwc[:, :2]], 1)
        return gx, gc1, gc2, gW, gb


def hip_linear_rank2(x: torch.Tensor, lin, c1: torch.Tensor, c2: torch.Tensor) -> torch.Tensor:
    """Linear(cat([x, c1[..., None], c2[..., None]], -1)) with nn.Linear ``lin`` [N, D + 2]:
    the stream GEMM with rank-1 epilogue terms (bf16 out) when D = 384 and N % 64 == 0 and the
    dW kernel's shapes fit (N % 128 == 0), else the f32 torch form."""
    D = x.shape[-1]
    W = lin.weight
    n_out = W.shape[0]
    if (train_dtype() == torch.float32 or D != 384 or n_out % 128 or lin.bias is None
            or os.environ.get("SNVRAG_TRAIN_NO_SG")):
        y = hip_linear(x, W[:, :D], lin.bias).float()
        return y + c1.unsqueeze(-1) * W[:, D] + c2.unsqueeze(-1) * W[:, D + 1]
    return _HipLinearRank2.apply(x, c1, c2, W, lin.bias)


class _NbrMeanDrop(torch.autograd.Function):
    """The train-mode neighbour K-mean with the reference's per-unique-neighbour dropout
    (embedding_rag_dataset.py:404-417): K.nbr_mean_drop / nbr_mean_drop_bwd, differentiable in the
    token table W and the panel AF embedding Ar (the mask regenerated from its seed)."""

    @staticmethod
    def forward(ctx, W, Ar, inv, codes, n_sites, pe, p, seed):
        Wf, Arf = W.detach().float().contiguous(), Ar.detach().float().contiguous()
        out = K.nbr_mean_drop(inv, codes, n_sites, Wf, pe, Arf, p, seed)
        ctx.save_for_backward(inv, codes, Wf, pe, Arf)
        ctx.cfg = (n_sites, p, seed, W.dtype, Ar.dtype)
        return out

    @staticmethod
    def backward(ctx, g):
        inv, codes, Wf, pe, Arf = ctx.saved_tensors
        n_sites, p, seed, wdt, adt = ctx.cfg
        dW = torch.zeros_like(Wf)
        dAr = torch.zeros_like(Arf)
        K.nbr_mean_drop_bwd(g.contiguous(), inv, codes, n_sites, Wf, pe, Arf, p, seed, dW, dAr)
        return dW.to(wdt), dAr.to(adt), None, None, None, None, None, None


def nbr_mean_drop(W, Ar, inv, codes, n_sites: int, pe, p: float) -> torch.Tensor:
    """f32 [nq, L, D] neighbour means of the unique neighbours ``inv`` [nq, k] (int, < 0: none,
    codes [U, ld] u8) under dropout p: one fused HIP launch each way instead of the [U, L, D]
    embeddings, their dropout and a [nq, U] x [U, L D] product."""
    return _NbrMeanDrop.apply(W, Ar, inv.to(torch.int32).contiguous(), codes.contiguous(), int(n_sites),
                              pe.float().contiguous(), float(p), _drop_seed())


class _HipAddLayerNorm(torch.autograd.Function):
    """y = drop_o(LayerNorm(x + drop_r(r))) (r optional) in bf16 with f32 statistics
    (snvrag_ln_fwd_train / snvrag_ln_bwd): one pass each way instead of torch's f32 conversion +
    LN + grad kernels, the dropouts around the norm fused (counter-based masks, regenerated by
    the backward)."""

    @staticmethod
    def forward(ctx, x, r, weight, bias, eps, p_r, p_out, seed, slope_x=0.0, slope_r=0.0, handoff=None):
        ctx.handoff = handoff
        x = x.to(torch.bfloat16).contiguous()
        r = r.to(torch.bfloat16).contiguous() if r is not None else None
        y, s, stats = K.ln_fwd_train(x, r, weight.detach().float().contiguous(),
                                     bias.detach().float().contiguous(), eps, p_r, p_out, seed, slope_x, slope_r)
        if slope_r != 0.0:
            ctx.save_for_backward(s, stats, weight, r)
        else:
            ctx.save_for_backward(s, stats, weight)
        ctx.has_r = r is not None
        ctx.drop = (p_r, p_out, seed)
        ctx.slopes = (slope_x, slope_r)
        ctx.params = (weight, bias)
        return y

    @staticmethod
    def backward(ctx, gy):
        s, stats, weight, *rp = ctx.saved_tensors
        p_r, p_out, seed = ctx.drop
        slope_x, slope_r = ctx.slopes
        w, b = ctx.params
        direct = _DIRECT_GRADS and _grad_buffer(w) is not None and _grad_buffer(b) is not None
        ds, dres, dg, db = K.ln_bwd(gy.to(torch.bfloat16).contiguous(), s, stats, weight.detach().float().contiguous(),
                                    p_r, p_out, seed, dg=w.grad if direct else None, db=b.grad if direct else None,
                                    slope_x=slope_x, slope_r=slope_r, r_pre=rp[0] if rp else None)
        dr = (dres if dres is not None else ds) if ctx.has_r else None
        dx = ds
        if ctx.handoff is not None and ctx.needs_input_grad[0]:
            ctx.handoff.g, dx = ds, None             # x's other consumer adds it (GradHandoff)
        if direct:
            return dx, dr, None, None, None, None, None, None, None, None, None
        return dx, dr, dg, db, None, None, None, None, None, None, None


def _drop_seed() -> int:
    return int(torch.randint(0, 2 ** 62, (1,)).item())


def hip_add_layernorm(x: torch.Tensor, r: Optional[torch.Tensor], ln, p_r: float = 0.0,
                      p_out: float = 0.0, act_x: float = 0.0, act_r: float = 0.0,
                      grad_to: Optional[GradHandoff] = None) -> torch.Tensor:
    """bf16 drop_o(LayerNorm(lrelu_x(x) + drop_r(lrelu_r(r)))) with the parameters of nn.LayerNorm
    ``ln`` (N % 8 == 0, N <= 2048); p_r / p_out: dropout on the residual operand / the output
    (training; the masks are a counter-based hash of a seed from torch's RNG); act_x / act_r:
    LeakyReLU slopes (0: none) fused into the norm (act_x only without a residual).  ``grad_to``:
    x's gradient is handed to x's other consumer (a ``hip_linear(x, ..., grad_from=...)`` upstream
    of ``r``) instead of being returned.  f32 parity mode: torch's f32 LeakyReLU, LayerNorm and
    F.dropout (no handoff: autograd adds the gradients)."""
    if train_dtype() == torch.float32:
        xx = torch.nn.functional.leaky_relu(x.float(), act_x) if act_x else x.float()
        rr = r.float() if r is not None else None
        if rr is not None and act_r:
            rr = torch.nn.functional.leaky_relu(rr, act_r)
        if rr is not None and p_r > 0:
            rr = torch.nn.functional.dropout(rr, p_r, True)
        s = xx + rr if rr is not None else xx
        y = torch.nn.functional.layer_norm(s, (s.shape[-1],), ln.weight, ln.bias, ln.eps)
        return torch.nn.functional.dropout(y, p_out, True) if p_out > 0 else y
    assert not (act_x and r is not None), "act_x is for a norm without a residual"
    seed = _drop_seed() if (p_r > 0 or p_out > 0) else 0
    assert grad_to is None or (r is not None and not act_x), "the handoff is for x of LN(x + r)"
    return _HipAddLayerNorm.apply(x, r, ln.weight, ln.bias, ln.eps, float(p_r), float(p_out), seed,
                                  float(act_x), float(act_r), grad_to)


class _HipAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, nseq, L, heads, dh, p, seed):
        qkv = qkv.contiguous()
        out, lse = K.attention_train_fwd(qkv, nseq, L, heads, dh, p, seed)
        ctx.save_for_backward(qkv, out, lse)
        ctx.shape = (nseq, L, heads, dh, p, seed)
        return out

    @staticmethod
    def backward(ctx, gout):
        qkv, out, lse = ctx.saved_tensors
        nseq, L, heads, dh, p, seed = ctx.shape
        g = gout.to(torch.bfloat16).contiguous()
        return K.attention_bwd(qkv, out, g, lse, nseq, L, heads, dh, p, seed), None, None, None, None, None, None


def hip_attention(qkv: torch.Tensor, nseq: int, L: int, heads: int, dh: int, dropout_p: float = 0.0,
                  seed: Optional[int] = None) -> torch.Tensor:
    """softmax(q k^T / sqrt(dh)) v per (sequence, head); qkv [nseq*L, 3D] bf16 -> [nseq*L, D].
    ``dropout_p`` > 0: attention-probability dropout (attention.py:28-29); the keep mask is a
    counter-based hash of ``seed`` (drawn from torch's RNG when None), shared by the backward."""
    if train_dtype() == torch.float32:
        # parity mode: the unfused f32 softmax attention (attention.py:21-31) under torch autograd
        D = heads * dh
        q, k, v = qkv.float().view(nseq, L, 3, heads, dh).permute(2, 0, 3, 1, 4)
        p = torch.softmax((q @ k.transpose(-1, -2)) / dh ** 0.5, -1)
        if dropout_p > 0:
            p = torch.nn.functional.dropout(p, dropout_p, True)
        return (p @ v).permute(0, 2, 1, 3).reshape(nseq * L, D)
    if dropout_p > 0 and seed is None:
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    return _HipAttention.apply(qkv, nseq, L, heads, dh, float(dropout_p), int(seed or 0))


class _FocalLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, probs, labels, mask, gamma, weight):
        loss, grad = K.focal_loss(probs.detach(), labels, mask, gamma, weight)
        ctx.save_for_backward(grad)
        ctx.dtype = probs.dtype
        return loss[0]

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return (grad * g).to(ctx.dtype), None, None, None, None


def focal_loss(probs: torch.Tensor, labels: torch.Tensor, mask: torch.Tensor, gamma: float = 2.0,
               weight: float = 1.0) -> torch.Tensor:
    """weight * FocalLoss(gamma, reduction='sum')(probs[mask], labels[mask]) — main/optim_schedule.py:64-96."""
    return _FocalLoss.apply(probs, labels, mask, gamma, weight)


class _RagMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, W, Ar, idx, codes, n_sites, pe, L, tok0, tok1, sos, eos, counts):
        out = K.rag_mean(idx, codes, n_sites, W.detach().float().contiguous(), pe, Ar.detach().float().contiguous(),
                         L, train_dtype(), tok0=tok0, tok1=tok1, sos=sos, eos=eos, counts=counts)
        valid = idx >= 0
        nv = valid.sum(1)
        if counts is not None:
            al = counts[:, :n_sites].float()
        else:
            al = (codes[idx.clamp(min=0)][:, :, :n_sites].float() * valid[:, :, None]).sum(1)
        frac = al / nv.clamp(min=1)[:, None]                                 # [nq, n_sites]
        ctx.save_for_backward(frac, (nv > 0).float())
        ctx.meta = (n_sites, W.shape, tok0, tok1, sos, eos)
        return out

    @staticmethod
    def backward(ctx, g):
        frac, anyq = ctx.saved_tensors
        n, wshape, tok0, tok1, sos, eos = ctx.meta
        G = g.float()
        gW = torch.zeros(wshape, device=g.device, dtype=torch.float32)
        Gs = G[:, 1:1 + n]
        gW[tok1] += torch.einsum("qs,qsd->d", frac, Gs)
        gW[tok0] += torch.einsum("qs,qsd->d", anyq[:, None] * (1 - frac), Gs)
        gW[sos] += G[:, 0].sum(0)
        if n + 1 < G.shape[1]:
            gW[eos] += G[:, n + 1].sum(0)
        # <pad> positions: nn.Embedding(padding_idx=0) accumulates no gradient
        gAr = G.sum(0)
        return gW, gAr, None, None, None, None, None, None, None, None, None, None


def rag_mean_train(W: torch.Tensor, Ar: torch.Tensor, idx: torch.Tensor, codes: torch.Tensor, n_sites: int,
                   pe: torch.Tensor, L: int, tok0: int = 5, tok1: int = 6, sos: int = 2, eos: int = 3,
                   counts: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[nq, L, D] bf16 mean of the k neighbours' complete-token embeddings, differentiable in W and Ar
    (``counts``: the neighbours' per-site alt-allele counts, sharded panels)."""
    return _RagMean.apply(W, Ar, idx, codes, n_sites, pe, L, tok0, tok1, sos, eos, counts)
