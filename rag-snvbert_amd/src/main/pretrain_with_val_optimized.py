"""BERTTrainerWithValidationOptimized — the v18 training loop
(reference: src/main/pretrain_with_val_optimized.py:30-552), one process per GPU.

Per batch (pretrain_with_val_optimized.py:160-245):
  retrieval  ``rag_dataset.process_batch_retrieval`` (HBM token index, exact int8-MFMA kNN)
  forward    BERTFoundationModel in train mode (src/train_forward.py, HIP autograd nodes)
  loss       3*FL(h1) + 3*FL(h2) + 4*FL(gt) over the masked sites, / grad_accum_steps
  backward   autograd; gradients accumulate in place in one flat f32 buffer, whose
             buckets are all-reduced over RCCL as they complete (GradBucketer)
  step       every grad_accum_steps: device-side clip (max_norm 1.0) + fused Adam +
             bf16 mirror (FusedAdam), ScheduledOptim LR update
Metrics (losses, TP/FP/FN per class, rare/common split by MAF) accumulate on the device
and are read once per ``log_freq`` batches / per epoch — no per-batch host sync.

The compute dtype is bf16 with f32 master weights and f32 accumulation (the reference
uses fp16 autocast + GradScaler; bf16's exponent range needs no loss scaling).
"""

from __future__ import annotations

import csv
import os
import time
from typing import Dict, Optional

import numpy as np
import torch
import torch.distributed as dist

from .optim_schedule import DeviceConfusion, FocalLoss, ScheduledOptim
from .optimizer import FlatParams, FusedAdam, GradBucketer


class BERTTrainerWithValidationOptimized:
    def __init__(self, model, train_dataloader=None, val_dataloader=None, vocab=None, lr: float = 1e-4,
                 betas=(0.9, 0.999), weight_decay: float = 0.01, warmup_steps: int = 10000,
                 with_cuda: bool = True, cuda_devices=None, log_freq: int = 10, grad_accum_steps: int = 1,
                 focal_gamma: float = 2.0, use_recon_loss: bool = False, patience: int = 5,
                 val_metric: str = "f1", min_delta: float = 0.001, rare_threshold: float = 0.05,
                 output_csv: Optional[str] = None, max_grad_norm: float = 1.0, bucket_bytes: int = 32 << 20):
        if use_recon_loss:
            raise NotImplementedError("use_recon_loss=True (MSE between embedding stages) is not supported")
        self.device = next(model.parameters()).device
        self.model = model
        self.train_data, self.val_data, self.vocab = train_dataloader, val_dataloader, vocab
        self.flat = FlatParams(model.parameters())
        self.optim = FusedAdam(self.flat, lr=lr, betas=betas, weight_decay=weight_decay,
                               max_grad_norm=max_grad_norm)
        self.optim_schedule = ScheduledOptim(self.optim, n_warmup_steps=warmup_steps, init_lr=lr * 0.2, max_lr=lr)
        self.ddp = GradBucketer(self.flat, bucket_bytes)
        self.grad_accum_steps = grad_accum_steps
        self.accum_step = 0
        self.focal_gamma = focal_gamma
        self.hap_criterion = FocalLoss(gamma=focal_gamma, reduction="sum")
        self.gt_criterion = FocalLoss(gamma=focal_gamma, reduction="sum")
        self.log_freq = log_freq
        self.patience, self.val_metric, self.min_delta = patience, val_metric, min_delta
        self.best_val_metric = -np.inf if val_metric in ("f1", "accuracy") else np.inf
        self.epochs_no_improve = 0
        self.best_model_path = None
        self.rare_threshold = rare_threshold
        self.output_csv = output_csv
        self.epoch_metrics = []
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.rag_train_dataset = getattr(train_dataloader, "dataset", None) if train_dataloader else None
        self.rag_val_dataset = getattr(val_dataloader, "dataset", None) if val_dataloader else None
        self.embedding_layer = model.bert.embedding
        self.rag_k = 1
        self.last_step_ms = None

    # ------------------------------------------------------------------ batch --
    def to_device(self, data: Dict) -> Dict:
        out = {}
        for k, v in data.items():
            out[k] = v.to(self.device, non_blocking=True) if torch.is_tensor(v) else v
        return out

    def loss(self, output, data) -> torch.Tensor:
        masks = data["mask"].bool()
        w = 1.0 / self.grad_accum_steps
        l1 = self.hap_criterion(output[0], data["hap_1_label"], masks, 3.0 * w)
        l2 = self.hap_criterion(output[1], data["hap_2_label"], masks, 3.0 * w)
        lg = self.gt_criterion(output[2], data["gt_label"], masks, 4.0 * w)
        return l1 + l2 + lg, (l1, l2, lg)

    def train_step(self, data: Dict) -> torch.Tensor:
        """One micro-batch: retrieval, forward, loss, backward (+ optimizer step on the last
        micro-batch of an accumulation group).  Returns the device loss (no sync)."""
        ds = self.rag_train_dataset
        # train mode BEFORE retrieval (pretrain_with_val_optimized.py:127): after validate() the
        # model is in eval mode, and retrieval in eval mode would return detached means
        self.model.train()
        if ds is not None and hasattr(ds, "process_batch_retrieval"):
            data = ds.process_batch_retrieval(data, self.embedding_layer, self.device, k_retrieve=self.rag_k)
        data = self.to_device(data)
        last = (self.accum_step + 1) % self.grad_accum_steps == 0
        self.ddp.enabled = last
        output = self.model(data)
        total, parts = self.loss(output, data)
        total.backward()
        self.accum_step += 1
        if last:
            scale = self.ddp.finish()
            self.optim.step(grad_scale=scale)
            self.optim_schedule.step()
            self.optim.zero_grad()
            self.accum_step = 0
        self._last = (output, data, parts)
        return total.detach()

    # ------------------------------------------------------------------ epoch --
    def train(self, epoch: int):
        return self._run_epoch(epoch, self.train_data, train=True)

    def validate(self, epoch: int):
        return self._run_epoch(epoch, self.val_data, train=False)

    def _run_epoch(self, epoch: int, dataloader, train: bool = True) -> Dict:
        dev = self.device
        loss_sum = torch.zeros(3, device=dev)
        hap, gt = DeviceConfusion(2, dev), DeviceConfusion(4, dev)
        rare, common = DeviceConfusion(2, dev), DeviceConfusion(2, dev)
        n_batches = 0
        t0 = time.perf_counter()
        for i, data in enumerate(dataloader):
            if train:
                self.train_step(data)
                output, data, parts = self._last
            else:
                ds = self.rag_val_dataset
                self.model.eval()
                with torch.no_grad():
                    if ds is not None and hasattr(ds, "process_batch_retrieval"):
                        data = ds.process_batch_retrieval(data, self.embedding_layer, dev, k_retrieve=self.rag_k)
                    data = self.to_device(data)
                    output = self.model(data)
                    _, parts = self.loss(output, data)
            with torch.no_grad():
                loss_sum += torch.stack([p.detach().float() for p in parts])
                m = data["mask"].bool()
                maf = torch.minimum(data["af"], 1 - data["af"])
                is_rare = (maf < self.rare_threshold) & m
                for k, lab in ((0, "hap_1_label"), (1, "hap_2_label")):
                    hap.update(output[k], data[lab], m)
                    rare.update(output[k], data[lab], m, is_rare)
                    common.update(output[k], data[lab], m, (~is_rare) & m)
                gt.update(output[2], data["gt_label"], m)
            n_batches += 1
            if train and self.log_freq and (i + 1) % self.log_freq == 0 and self.rank == 0:
                ls = (loss_sum / n_batches).tolist()
                print(f"EP_Train:{epoch} it {i + 1} loss h1 {ls[0]:.4f} h2 {ls[1]:.4f} gt {ls[2]:.4f} "
                      f"{(time.perf_counter() - t0) / (i + 1) * 1e3:.1f} ms/it", flush=True)
        torch.cuda.synchronize(dev) if dev.type == "cuda" else None
        elapsed = time.perf_counter() - t0
        ls = (loss_sum / max(n_batches, 1)).tolist()
        res = {"epoch": epoch, "mode": "train" if train else "val", "hap_loss": ls[0] + ls[1], "gt_loss": ls[2],
               "hap_f1": hap.f1(), "gt_f1": gt.f1(), "rare_f1": rare.f1(), "common_f1": common.f1(),
               "batches": n_batches, "sec": elapsed}
        self.epoch_metrics.append(res)
        if self.rank == 0:
            print(f"{'Train' if train else 'Val'} epoch {epoch}: " +
                  " ".join(f"{k}={v:.4f}" if isinstance(v, float) else f"{k}={v}" for k, v in res.items()),
                  flush=True)
            if self.output_csv:
                new = not os.path.exists(self.output_csv)
                with open(self.output_csv, "a", newline="") as f:
                    w = csv.DictWriter(f, fieldnames=list(res))
                    if new:
                        w.writeheader()
                    w.writerow(res)
        return res

    # ------------------------------------------------------------- checkpoint --
    def save(self, epoch: int, file_path: str = "output/bert_trained.model") -> str:
        """state_dict checkpoint (+ optimizer/schedule state) instead of the reference's pickled
        module (pretrain_with_val_optimized.py:524-552): loadable with weights_only=True."""
        path = f"{file_path}.ep{epoch}"
        if self.rank == 0:
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
            torch.save({"model": {k: v.detach().cpu() for k, v in self.model.state_dict().items()},
                        "optim": self.optim.state_dict(),
                        "schedule_steps": self.optim_schedule.n_current_steps, "epoch": epoch}, path)
        return path

    def load(self, path: str) -> int:
        ck = torch.load(path, map_location="cpu", weights_only=True)
        sd = ck["model"] if "model" in ck else ck
        sd = {k[7:] if k.startswith("module.") else k: v for k, v in sd.items()}
        self.model.load_state_dict(sd)
        self.flat.sync_mirror()
        if "optim" in ck:
            self.optim.load_state_dict(ck["optim"])
            self.optim_schedule.n_current_steps = int(ck.get("schedule_steps", 0))
        return int(ck.get("epoch", 0))

    def should_stop_early(self, val_res: Dict) -> bool:
        key = {"f1": "hap_f1", "accuracy": "hap_f1", "loss": "hap_loss"}.get(self.val_metric, "hap_f1")
        v = val_res[key]
        better = v > self.best_val_metric + self.min_delta if self.val_metric != "loss" else \
            v < self.best_val_metric - self.min_delta
        if better:
            self.best_val_metric, self.epochs_no_improve = v, 0
            return False
        self.epochs_no_improve += 1
        return self.epochs_no_improve >= self.patience
