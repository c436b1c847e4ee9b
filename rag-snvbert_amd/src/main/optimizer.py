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
  GradBucketer  DDP gradient exchange: contiguous buckets of the flat gradient buffer
                (parameters laid out in reverse registration order, so buckets fill in
                backward order) are all-reduced (SUM) asynchronously (RCCL over xGMI on the
                GPU, gloo in the CPU tests) once every parameter in them is final, in one
                bucket order on every rank, overlapping the rest of the backward pass.
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
        self.sq_ws = torch.empty(int(K.N.lib().snvrag_sqnorm_ws_bytes()) // 4, device=flat.flat.device,
                                 dtype=torch.float32)      # the norm's per-block partials (this optimizer's own)
        self.step_count = 0
        self.param_groups = [{"lr": lr}]          # ScheduledOptim writes the LR here

    def zero_grad(self) -> None:
        self.fp.zero_grad()

    def step(self, grad_scale: float = 1.0) -> None:
        self.step_count += 1
        lr = float(self.param_groups[0]["lr"])
        if self.max_grad_norm and self.max_grad_norm > 0:
            self.K.sqnorm(self.fp.grad, self.sq, ws=self.sq_ws)
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
    """Bucketed asynchronous all-reduce of FlatParams.grad (DDP gradient exchange).

    Readiness: a parameter reports ONCE per backward, from its post-accumulate hook.  Autograd
    runs a leaf's AccumulateGrad node once per backward, after every use of the parameter has
    run its backward — also for the parameters whose HIP backward adds dW / db straight into
    the flat buffer (``autograd_ops.direct_weight_grads``: the node then sees an undefined
    gradient and adds nothing, and the hook still fires).  A parameter used several times in a
    step (the AF MLP runs for the queries and once per neighbour window group) therefore reports
    after its LAST contribution has been enqueued, never earlier.  A second report in one step
    is an error.

    Launch order: bucket b is all-reduced once all of its parameters reported AND buckets
    0..b-1 were launched — the same order (0, 1, 2, ...) on every rank whatever order the
    rank's graph finished its parameters in (a rank with more neighbour window groups finishes
    the embedding bucket later; RCCL needs the collectives in one order everywhere).  Buckets
    with parameters that got no gradient this step are launched by ``finish`` (in order).

    Reduction: SUM.  The reference trains with nn.DataParallel (pretrain_with_val_optimized.py:
    59-65): one summed focal loss over the whole global batch (:215-233) and ONE gradient, which
    is clipped and stepped (:235-245).  With the global batch split over ranks, the sum of the
    ranks' gradients of their summed losses IS that gradient; ``finish`` returns grad scale 1.
    ``average=True`` gives torch-DDP averaging (scale 1 / world) instead."""

    def __init__(self, flat: FlatParams, bucket_bytes: int = 32 << 20, group=None, always: bool = False,
                 average: bool = False):
        """``always``: run the collectives even in a world of one (the RCCL smoke test)."""
        self.fp = flat
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.active = self.world > 1 or (always and dist.is_initialized())
        self.average = average
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
        self.ready: List[set] = [set() for _ in self.buckets]
        self.next_launch = 0
        self.handles: Dict[int, object] = {}
        self.staged: Dict[int, torch.Tensor] = {}
        self.enabled = True
        self.trace: Optional[list] = None          # tests: [(bucket, frozenset(ready params))] per launch
        self._hooks = []
        if self.active:
            self._stage = dist.get_backend(group) == "gloo" and flat.grad.is_cuda
            for i, p in enumerate(flat.params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))

    def _close(self, idxs, start, end):
        if idxs:
            self.buckets.append(list(idxs))
            self.bounds.append((start, end))

    def _make_hook(self, i):
        def hook(_p):
            if not self.enabled:
                return
            b = self.owner[i]
            if i in self.ready[b]:
                raise RuntimeError(f"GradBucketer: parameter {i} reported ready twice in one backward")
            self.ready[b].add(i)
            while self.next_launch < len(self.buckets) and \
                    len(self.ready[self.next_launch]) == len(self.buckets[self.next_launch]):
                self._launch(self.next_launch)
        return hook

    def _launch(self, b):
        assert b == self.next_launch and b not in self.handles
        if self.trace is not None:
            self.trace.append((b, frozenset(self.ready[b])))
        s, e = self.bounds[b]
        if self._stage:
            # gloo (the CPU-collective tests with the ranks' tensors on a GPU): through the host
            host = self.fp.grad[s:e].cpu()
            self.handles[b] = dist.all_reduce(host, group=self.group, async_op=True)
            self.staged[b] = host
        else:
            self.handles[b] = dist.all_reduce(self.fp.grad[s:e], group=self.group, async_op=True)
        self.next_launch += 1

    def finish(self) -> float:
        """Launch the buckets not launched yet (parameters without a gradient this step), in
        order, wait for all; returns the grad scale FusedAdam applies (1: SUM, see class doc)."""
        if self.active:
            while self.next_launch < len(self.buckets):
                self._launch(self.next_launch)
            for b in sorted(self.handles):
                self.handles[b].wait()
                if b in self.staged:
                    s, e = self.bounds[b]
                    self.fp.grad[s:e].copy_(self.staged[b])
        self.handles.clear()
        self.staged.clear()
        self.ready = [set() for _ in self.buckets]
        self.next_launch = 0
        return 1.0 / self.world if self.average else 1.0
