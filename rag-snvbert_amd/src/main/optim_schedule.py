"""Loss, LR schedule and metrics of the v18 trainer (reference: src/main/optim_schedule.py).

  FocalLoss       optim_schedule.py:49-96 — forward AND backward on the device
                  (snvrag_focal_loss); the loss "inputs" are the heads' softmax
                  probabilities, re-softmaxed inside exactly as the reference does.
  ScheduledOptim  optim_schedule.py:11-46 — linear warmup init_lr -> max_lr, then
                  inverse-square-root decay; writes param_groups[0]['lr'].
  cal_acc/cal_pr  optim_schedule.py:99-109, :167-203 — host versions (API parity) and
                  ``DeviceConfusion``: the same TP/FP/FN counts accumulated on the GPU
                  without a per-batch device->host copy.
"""

from __future__ import annotations

import torch

from .. import kernels as K
from ..autograd_ops import focal_loss


class FocalLoss(torch.nn.Module):
    def __init__(self, gamma: float = 2.0, alpha=None, reduction: str = "sum", ignore_index=None):
        super().__init__()
        if alpha is not None or ignore_index is not None or reduction != "sum":
            raise NotImplementedError("the v18 trainer uses FocalLoss(gamma, reduction='sum') "
                                      "(pretrain_with_val_optimized.py:87-88)")
        self.gamma = gamma

    def forward(self, inputs: torch.Tensor, targets: torch.Tensor, mask: torch.Tensor = None,
                weight: float = 1.0) -> torch.Tensor:
        """FL over rows where ``mask`` (default: all rows); ``weight`` scales loss and gradient."""
        if mask is None:
            mask = torch.ones(targets.shape, dtype=torch.bool, device=targets.device)
        return focal_loss(inputs, targets, mask, self.gamma, weight)


class ScheduledOptim:
    def __init__(self, optimizer, n_warmup_steps: int, init_lr: float = 1e-5, max_lr: float = 5e-5):
        self._optimizer = optimizer
        self.n_warmup_steps = n_warmup_steps
        self.n_current_steps = 0
        self.init_lr, self.max_lr = init_lr, max_lr

    def step(self) -> None:
        self.n_current_steps += 1
        lr = self._get_lr_scale()
        for g in self._optimizer.param_groups:
            g["lr"] = lr

    def zero_grad(self) -> None:
        self._optimizer.zero_grad()

    def _get_lr_scale(self) -> float:
        if self.n_current_steps <= self.n_warmup_steps:
            return (self.max_lr - self.init_lr) / self.n_warmup_steps * self.n_current_steps + self.init_lr
        return self.max_lr * (self.n_warmup_steps ** 0.5) * (self.n_current_steps ** -0.5)


def cal_acc(pred: torch.Tensor, label: torch.Tensor, mask: torch.Tensor):
    p = pred.argmax(-1).flatten()
    m = mask.flatten().bool()
    return int((p.eq(label.flatten()) & m).sum().item()), int(m.sum().item())


def cal_pr(pred: torch.Tensor, label: torch.Tensor, mask: torch.Tensor, num_classes: int):
    p = pred.argmax(-1).flatten()
    lab = label.flatten()
    m = mask.flatten().bool()
    p, lab = p[m], lab[m]
    out = {k: torch.zeros(num_classes, dtype=torch.long) for k in ("tp", "fp", "fn")}
    for c in range(num_classes):
        out["tp"][c] += int(((p == c) & (lab == c)).sum())
        out["fp"][c] += int(((p == c) & (lab != c)).sum())
        out["fn"][c] += int(((p != c) & (lab == c)).sum())
    return out


class DeviceConfusion:
    """TP/FP/FN per class accumulated on the device (cal_pr without the D2H copy)."""

    def __init__(self, num_classes: int, device):
        self.C = num_classes
        self.counts = torch.zeros(3, num_classes, dtype=torch.int64, device=device)

    def update(self, probs, labels, mask, mask2=None) -> None:
        K.confusion(probs.detach(), labels, mask, self.counts, mask2)

    def host(self):
        c = self.counts.cpu()
        return {"tp": c[0], "fp": c[1], "fn": c[2]}

    def f1(self) -> float:
        c = self.counts.double().cpu()
        tp, fp, fn = c[0], c[1], c[2]
        prec = tp / (tp + fp).clamp(min=1)
        rec = tp / (tp + fn).clamp(min=1)
        f1 = 2 * prec * rec / (prec + rec).clamp(min=1e-12)
        return float(f1.mean())
