"""CPU restatement (numpy) of the reference's training-step arithmetic — TEST
INFRASTRUCTURE ONLY (imported by tests/ and never by the product path).

  focal_loss   main/optim_schedule.py:64-96 (FocalLoss.forward, reduction='sum', softmax
               applied to the inputs, eps 1e-10) and its analytic derivative w.r.t. the
               inputs.  Pinned by tests/golden/focal.npz (reference autograd).
  adam_step    torch.optim.Adam (pretrain_with_val_optimized.py:73-74) with
               clip_grad_norm_(max_norm) (:239-241): L2 weight decay in the gradient,
               bias-corrected moments.
  lr_schedule  ScheduledOptim._get_lr_scale (optim_schedule.py:33-38).
  confusion    cal_pr (optim_schedule.py:167-203): per-class TP/FP/FN of argmax predictions
               over the masked rows.
"""

from __future__ import annotations

import numpy as np


def focal_loss(x: np.ndarray, y: np.ndarray, mask: np.ndarray, gamma: float = 2.0):
    """(sum of FL over rows with mask, dFL/dx [M, C]) in float64."""
    x = np.asarray(x, np.float64)
    s = np.exp(x - x.max(-1, keepdims=True))
    s /= s.sum(-1, keepdims=True)
    rows = np.arange(len(y))
    pt = s[rows, y]
    q = 1.0 - pt
    lp = np.log(pt + 1e-10)
    loss = -(q ** gamma) * lp
    dpt = (gamma * q ** (gamma - 1) * lp if gamma != 0 else 0.0) - q ** gamma / (pt + 1e-10)
    onehot = np.zeros_like(s)
    onehot[rows, y] = 1.0
    grad = (dpt * pt)[:, None] * (onehot - s)
    m = np.asarray(mask, bool)
    grad[~m] = 0.0
    return float(loss[m].sum()), grad


def adam_step(p, g, m, v, *, lr, betas, eps, weight_decay, step, grad_scale=1.0, max_norm=0.0):
    p, g, m, v = (np.asarray(a, np.float64).copy() for a in (p, g, m, v))
    g = g * grad_scale
    if max_norm > 0:
        norm = np.sqrt((g ** 2).sum())
        g = g * min(1.0, max_norm / (norm + 1e-6))
    g = g + weight_decay * p
    b1, b2 = betas
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    p = p - (lr / bc1) * m / (np.sqrt(v) / np.sqrt(bc2) + eps)
    return p, m, v


def lr_schedule(step: int, warmup: int, init_lr: float, max_lr: float) -> float:
    if step <= warmup:
        return (max_lr - init_lr) / warmup * step + init_lr
    return max_lr * (warmup ** 0.5) * (step ** -0.5)


def confusion(probs: np.ndarray, labels: np.ndarray, mask: np.ndarray, num_classes: int) -> np.ndarray:
    """int64 [3, C] = (tp, fp, fn) per class over rows with mask (argmax: first maximum)."""
    p = np.asarray(probs).reshape(-1, num_classes).argmax(-1)
    y = np.asarray(labels).reshape(-1)
    m = np.asarray(mask).reshape(-1).astype(bool)
    p, y = p[m], y[m]
    out = np.zeros((3, num_classes), np.int64)
    for c in range(num_classes):
        out[0, c] = ((p == c) & (y == c)).sum()
        out[1, c] = ((p == c) & (y != c)).sum()
        out[2, c] = ((p != c) & (y == c)).sum()
    return out
