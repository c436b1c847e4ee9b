"""Flat-buffer optimizer state, fused Adam on the device, and bucketed gradient all-reduce.

Replaces the trainer step of main/pretrain_with_val_optimized.py:235-245
(``scaler.backward``, ``clip_grad_norm_(max_norm=1.0)``, fused ``torch.optim.Adam``) and
the data-parallel wrapper (``nn.DataParallel`` there; one process per GPU here):

  FlatParams    every trainable parameter becomes a view into ONE f32 buffer, its
                ``.grad`` a view into one f32 gradient buffer (autograd accumulates in
                place), plus a bf16 mirror the MFMA GEMMs read (autograd_ops.bf16_of).
                Offsets are padded to 64 elements (16-byte aligned bf16/f32 views).
  FusedAdam     snvrag_sqnorm + snvrag_adam_step: clip coefficient computed on the
                device, Adam update and the bf16 mirror in one pass over the buffer —
                no host synchronisation in the step.
  GradBucketer  DDP gradient averaging: contiguous buckets of the flat gradient buffer
                (parameters laid out in reverse registration order, so buckets fill in
                backward order) are all-reduced asynchronously (RCCL over xGMI on the
                GPU, gloo in the CPU tests) as soon as their last gradient is
                accumulated, overlapping the rest of the backward pass.
"""

from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from .. import autograd_ops

ALIGN = 64


class FlatParams:
    def __init__(self, params, mirror: bool = True):
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad][::-1]
        if not self.params:
            raise ValueError("no trainable parameters")
        dev = self.params[0].device
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.numel = off
        self.flat = torch.zeros(off, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(off, device=dev, dtype=torch.float32)
        self.bf16 = torch.zeros(off, device=dev, dtype=torch.bfloat16) if mirror and dev.type == "cuda" else None
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            self.flat[o:o + n].copy_(p.detach().reshape(-1))
            p.data = self.flat[o:o + n].view_as(p)
            p.grad = self.grad[o:o + n].view_as(p)
        self.sync_mirror()

    def view(self, buf: torch.Tensor, i: int) -> torch.Tensor:
        p, o = self.params[i], self.offsets[i]
        return buf[o:o + p.numel()].view_as(p)

    def sync_mirror(self) -> None:
        """Refresh the bf16 mirror from the f32 master (after load_state_dict or manual edits)."""
        if self.bf16 is None:
            return
        self.bf16.copy_(self.flat)
        for i, p in enumerate(self.params):
            autograd_ops.register_mirror(p, self.view(self.bf16, i))
        autograd_ops.weights_updated()

    def zero_grad(self) -> None:
        self.grad.zero_()
        for i, p in enumerate(self.params):
            if p.grad is None or p.grad.data_ptr() != self.view(self.grad, i).data_ptr():
                p.grad = self.view(self.grad, i)


class FusedAdam:
    """torch.optim.Adam semantics (L2 weight decay in the gradient, bias correction)."""

    def __init__(self, flat: FlatParams, lr: float = 1e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, max_grad_norm: float = 1.0):
        from .. import kernels as K
        self.K = K
        self.fp = flat
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.max_grad_norm = max_grad_norm
        self.m = torch.zeros_like(flat.flat)
        self.v = torch.zeros_like(flat.flat)
        self.sq = torch.zeros(1, device=flat.flat.device, dtype=torch.float32)
        self.step_count = 0
        self.param_groups = [{"lr": lr}]          # ScheduledOptim writes the LR here

    def zero_grad(self) -> None:
        self.fp.zero_grad()

    def step(self, grad_scale: float = 1.0) -> None:
        self.step_count += 1
        lr = float(self.param_groups[0]["lr"])
        if self.max_grad_norm and self.max_grad_norm > 0:
            self.K.sqnorm(self.fp.grad, self.sq)
        self.K.adam_step(self.fp.flat, self.fp.grad, self.m, self.v, lr=lr, betas=self.betas, eps=self.eps,
                         weight_decay=self.weight_decay, step=self.step_count, grad_scale=grad_scale,
                         max_norm=self.max_grad_norm or 0.0, sq=self.sq if self.max_grad_norm else None,
                         p_bf16=self.fp.bf16)
        autograd_ops.weights_updated()

    def grad_norm(self, grad_scale: float = 1.0) -> torch.Tensor:
        """L2 norm of the (scaled) gradient of the last step (device tensor)."""
        return self.sq.sqrt() * grad_scale

    def state_dict(self) -> Dict:
        return {"m": self.m.cpu(), "v": self.v.cpu(), "step": self.step_count, "lr": self.param_groups[0]["lr"],
                "betas": self.betas, "eps": self.eps, "weight_decay": self.weight_decay}

    def load_state_dict(self, sd: Dict) -> None:
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.step_count = int(sd["step"])
        self.param_groups[0]["lr"] = sd["lr"]


class GradBucketer:
    """Bucketed asynchronous all-reduce (SUM) of FlatParams.grad; averaging is folded into
    FusedAdam's grad_scale (1 / world)."""

    def __init__(self, flat: FlatParams, bucket_bytes: int = 32 << 20, group=None, always: bool = False):
        """``always``: run the collectives even in a world of one (the RCCL smoke test)."""
        self.fp = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.active = self.world > 1 or (always and dist.is_initialized())
        self.buckets: List[List[int]] = []        # param indices (flat order)
        self.bounds: List[tuple] = []
        cur, start, size = [], 0, 0
        for i, p in enumerate(flat.params):
            nbytes = p.numel() * 4
            if cur and size + nbytes > bucket_bytes:
                self._close(cur, start, flat.offsets[i])
                cur, start, size = [], flat.offsets[i], 0
            cur.append(i)
            size += nbytes
        self._close(cur, start, flat.numel)
        self.owner = {}
        for b, idxs in enumerate(self.buckets):
            for i in idxs:
                self.owner[i] = b
        self.pending = [0] * len(self.buckets)
        self.handles: Dict[int, object] = {}
        self.enabled = True
        self._hooks = []
        if self.active:
            for i, p in enumerate(flat.params):
                hook = self._make_hook(i)
                self._hooks.append(p.register_post_accumulate_grad_hook(hook))
                p._snv_grad_ready = hook           # gradients accumulated in place by the HIP ops

    def _close(self, idxs, start, end):
        if idxs:
            self.buckets.append(list(idxs))
            self.bounds.append((start, end))

    def _make_hook(self, i):
        def hook(_p):
            if not self.enabled:
                return
            b = self.owner[i]
            self.pending[b] += 1
            if self.pending[b] == len(self.buckets[b]) and b not in self.handles:
                self._launch(b)
        return hook

    def _launch(self, b):
        s, e = self.bounds[b]
        self.handles[b] = dist.all_reduce(self.fp.grad[s:e], group=self.group, async_op=True)

    def finish(self) -> float:
        """Wait for every bucket (launching those whose parameters got no gradient this step);
        returns the grad scale that averages over ranks."""
        if self.active:
            for b in range(len(self.buckets)):
                if b not in self.handles:
                    self._launch(b)
            for b in sorted(self.handles):
                self.handles[b].wait()
        self.handles.clear()
        self.pending = [0] * len(self.buckets)
        return 1.0 / self.world
