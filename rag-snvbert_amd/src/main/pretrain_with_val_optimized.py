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

Several ranks (one process per GPU) are one data-parallel trainer over a global batch of
world x per-rank batch, the reference's nn.DataParallel (:59-65) without the replica
scatter/gather:
  * gradients: SUM all-reduce (GradBucketer) — the gradient of the reference's one summed loss
    over the global batch;
  * epoch metrics: the loss sums and every TP/FP/FN count are summed over ranks before the CSV
    row, ``is_best`` and early stopping, so they describe the WHOLE epoch (:362-372, :490-500);
    the batch count is the number of global steps (equal on every rank);
  * early stopping: decided on those global counts and broadcast from rank 0, so every rank
    leaves the epoch loop together;
  * BatchNorm running statistics (PositionFeatModule, fusion.py:317-332): each rank advances its
    own from its batches (batch statistics of its chunk, as a DataParallel replica does); at
    the end of every training epoch rank 0's buffers are broadcast — DataParallel keeps only
    device 0's updates too — so validation and checkpoints use the same statistics everywhere.

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

from .. import autograd_ops
from .optim_schedule import DeviceConfusion, FocalLoss, ScheduledOptim
from .optimizer import FlatParams, FusedAdam, GradBucketer


MIN_RECON_LOSS = 0.01        # pretrain_with_val_optimized.py:18


def recon_mse(a: torch.Tensor, b: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """nn.MSELoss()(a[mask], b[mask]) in f32: the mean of the squared differences over the
    masked sites' features.  An empty mask gives 0 (the reference's NaN fails both threshold
    comparisons the same way, and 0 keeps NaN out of the unselected branch's gradient)."""
    d = (a.float() - b.float()) * mask.unsqueeze(-1)
    n = (mask.sum() * a.shape[-1]).clamp(min=1)
    return d.pow(2).sum() / n


def _sum_over_ranks(x: torch.Tensor) -> torch.Tensor:
    """all_reduce(SUM) of a small metric tensor (through the host for gloo)."""
    if dist.get_backend() == "gloo" and x.is_cuda:
        h = x.cpu()
        dist.all_reduce(h)
        return h.to(x.device)
    dist.all_reduce(x)
    return x


class BERTTrainerWithValidationOptimized:
    def __init__(self, model, train_dataloader=None, val_dataloader=None, vocab=None, lr: float = 1e-4,
                 betas=(0.9, 0.999), weight_decay: float = 0.01, warmup_steps: int = 10000,
                 with_cuda: bool = True, cuda_devices=None, log_freq: int = 10, grad_accum_steps: int = 1,
                 focal_gamma: float = 2.0, use_recon_loss: bool = False, patience: int = 5,
                 val_metric: str = "f1", min_delta: float = 0.001, rare_threshold: float = 0.05,
                 output_csv: Optional[str] = None, max_grad_norm: float = 1.0, bucket_bytes: int = 32 << 20):
        self.use_recon_loss = bool(use_recon_loss)
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
        # early stopping always monitors the validation hap F1 (should_stop_early), higher is better;
        # the reference starts at +inf for val_metric='loss', after which nothing ever improves
        self.best_val_metric = -np.inf
        self.epochs_no_improve = 0
        self.best_model_path = None
        self.rare_threshold = rare_threshold
        self.output_csv = output_csv
        self.epoch_metrics = []
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.rag_train_dataset = getattr(train_dataloader, "dataset", None) if train_dataloader else None
        self.rag_val_dataset = getattr(val_dataloader, "dataset", None) if val_dataloader else None
        self.embedding_layer = model.bert.embedding
        self.rag_k = 1
        self.last_step_ms = None

    # ------------------------------------------------------------------ batch --
    def to_device(self, data: Dict) -> Dict:
        """Batch tensors to the device without a host sync (pageable ones through pinned staging)."""
        from ..dataset.embedding_rag_dataset import h2d
        dev = torch.device(self.device)
        out = {}
        for k, v in data.items():
            out[k] = h2d(v, dev) if torch.is_tensor(v) else v
        return out

    def loss(self, output, data) -> torch.Tensor:
        """(3 FL(h1) + 3 FL(h2) + 4 FL(gt)) / grad_accum_steps over the masked sites
        (pretrain_with_val_optimized.py:215-233) and the three unweighted focal losses the
        reference's metrics accumulate (:312-313).

        ``use_recon_loss`` (:219-228): the MSE between the raw embeddings (outputs 3, 4) and the
        encoder outputs (5, 6) at the masked sites, nn.MSELoss (mean over sites x features);
        when both exceed MIN_RECON_LOSS = 0.01 the total becomes 0.2 FL(h1) + 0.2 FL(h2) +
        0.3 FL(gt) + 0.15 MSE1 + 0.15 MSE2, else the plain weighting.  The branch is decided on
        the device (torch.where), without the reference's host sync on the comparison."""
        masks = data["mask"].bool()
        w = 1.0 / self.grad_accum_steps
        l1 = self.hap_criterion(output[0], data["hap_1_label"], masks)
        l2 = self.hap_criterion(output[1], data["hap_2_label"], masks)
        lg = self.gt_criterion(output[2], data["gt_label"], masks)
        total = 3.0 * l1 + 3.0 * l2 + 4.0 * lg
        if self.use_recon_loss:
            r1 = recon_mse(output[3], output[5], masks)
            r2 = recon_mse(output[4], output[6], masks)
            alt = 0.2 * l1 + 0.2 * l2 + 0.3 * lg + 0.15 * r1 + 0.15 * r2
            total = torch.where((r1 > MIN_RECON_LOSS) & (r2 > MIN_RECON_LOSS), alt, total)
        return total * w, (l1, l2, lg)

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
        with autograd_ops.direct_weight_grads():
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
                is_rare = (maf < self.rare_threshold) & m          # :281-288
                for k, lab in ((0, "hap_1_label"), (1, "hap_2_label")):
                    hap.update(output[k], data[lab], m)
                    rare.update(output[k], data[lab], m, is_rare)
                    common.update(output[k], data[lab], m, (~is_rare) & m)
                gt.update(output[2], data["gt_label"], m)
            n_batches += 1
            if train and self.log_freq and i % self.log_freq == 0 and self.rank == 0:
                # _print_log (:335-360): ALT-class (class 1) haplotype precision / recall / F1
                c = hap.counts.float().cpu()
                p_, r_, f_ = self.calculate_metrics(c[0], c[1], c[2])
                ls = (loss_sum / n_batches).tolist()
                print(f"EP_Train:{epoch} it {i} Precision {p_[1].item():.4f} Recall {r_[1].item():.4f} "
                      f"F1 {f_[1].item():.4f} avg_hap_loss {ls[0] + ls[1]:.4f} avg_gt_loss {ls[2]:.4f} "
                      f"{(time.perf_counter() - t0) / (i + 1) * 1e3:.1f} ms/it", flush=True)
        confs = (("hap", hap), ("gt", gt), ("rare", rare), ("common", common))
        if self.world > 1:
            # the whole epoch's metrics (:362-372): sum the loss sums and counts over ranks (f64
            # holds the integer counts exactly); batches = global steps, equal on every rank
            packed = torch.cat([loss_sum.double()] + [c.counts.double().reshape(-1) for _, c in confs] +
                               [torch.tensor([float(n_batches)], device=dev, dtype=torch.float64)])
            packed = _sum_over_ranks(packed)
            loss_sum = packed[:3].float()
            off = 3
            for _, c in confs:
                c.counts = packed[off:off + c.counts.numel()].round().long().view_as(c.counts)
                off += c.counts.numel()
            n_batches = int(round(packed[off].item() / self.world))
            if train:
                self.sync_buffers()
        torch.cuda.synchronize(dev) if dev.type == "cuda" else None
        elapsed = time.perf_counter() - t0
        ls = loss_sum.tolist()
        counts = {name: conf.counts.cpu() for name, conf in confs}
        row = self.metric_row(epoch, train, counts, ls[0] + ls[1], max(n_batches, 1))
        self.epoch_metrics.append(row)
        res = dict(row)
        for name, c in counts.items():                         # eval_dict's tp / fp / fn (:132-154)
            res[f"{name}_tp"], res[f"{name}_fp"], res[f"{name}_fn"] = c[0], c[1], c[2]
        gt_p, gt_r, gt_f1 = self.calculate_metrics(*counts["gt"].float())
        res.update(hap_loss=ls[0] + ls[1], gt_loss=ls[2], gt_f1=float(gt_f1.mean()), batches=n_batches, sec=elapsed)
        if self.rank == 0:
            print(f"{'Train' if train else 'Val'} epoch {epoch + 1}: " +
                  " ".join(f"{k}={v:.4f}" if isinstance(v, float) else f"{k}={v}" for k, v in row.items()) +
                  f" gt_avg_f1={res['gt_f1']:.4f} {elapsed:.1f}s", flush=True)
            if self.output_csv:
                self._save_epoch_metrics(row)
        return res

    def sync_buffers(self) -> None:
        """Broadcast rank 0's buffers (the BatchNorm running statistics) to every rank — the
        statistics DataParallel keeps (device 0's replica is the module)."""
        if self.world <= 1:
            return
        for b in self.model.buffers():
            if dist.get_backend() == "gloo" and b.is_cuda:
                h = b.detach().cpu()
                dist.broadcast(h, 0)
                b.data.copy_(h)
            else:
                dist.broadcast(b.data, 0)

    # ------------------------------------------------------------ metrics --
    @staticmethod
    def calculate_metrics(tp: torch.Tensor, fp: torch.Tensor, fn: torch.Tensor):
        """Per-class precision, recall, F1 (pretrain_with_val_optimized.py:483-488), f32."""
        tp, fp, fn = tp.float(), fp.float(), fn.float()
        precision = tp / (tp + fp + 1e-10)
        recall = tp / (tp + fn + 1e-10)
        f1 = 2 * precision * recall / (precision + recall + 1e-10)
        return precision, recall, f1

    def metric_row(self, epoch: int, train: bool, counts: Dict[str, torch.Tensor], hap_loss_sum: float,
                   num_batches: int, correct: Optional[int] = None, total: Optional[int] = None) -> Dict:
        """The reference's per-epoch CSV row (:424-481): ALT-class (index 1) metrics overall and
        split into rare (MAF < rare_threshold) / common sites; ``counts[name]`` = [tp; fp; fn] per
        class; accuracy = correct / masked haplotype sites (cal_acc, optim_schedule.py:99-109) —
        by default from the counts (an argmax call is right iff it is a TP of its label's class,
        and every masked site is a TP or an FN of its label's class)."""
        c = counts["hap"]
        hp, hr, hf = self.calculate_metrics(c[0], c[1], c[2])
        rp, rr, rf = self.calculate_metrics(*counts["rare"])
        cp, cr, cf = self.calculate_metrics(*counts["common"])
        if correct is None:
            correct, total = int(c[0].sum()), int((c[0] + c[2]).sum())
        return {"epoch": epoch + 1, "mode": "train" if train else "val",
                "loss": hap_loss_sum / num_batches,
                "accuracy": correct / total if total else float("nan"),
                "overall_f1": hf[1].item(), "overall_precision": hp[1].item(), "overall_recall": hr[1].item(),
                "rare_f1": rf[1].item(), "rare_precision": rp[1].item(), "rare_recall": rr[1].item(),
                "common_f1": cf[1].item(), "common_precision": cp[1].item(), "common_recall": cr[1].item()}

    def _save_epoch_metrics(self, row: Dict) -> None:
        """Append ``row`` to output_csv, header on first write (:466-481)."""
        os.makedirs(os.path.dirname(self.output_csv) or ".", exist_ok=True)
        new = not os.path.exists(self.output_csv)
        with open(self.output_csv, "a", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(row))
            if new:
                w.writeheader()
            w.writerow(row)

    # ------------------------------------------------------------- checkpoint --
    def _checkpoint(self, epoch: int) -> Dict:
        ck = {"model": {k: v.detach().cpu() for k, v in self.model.state_dict().items()},
              "optim": self.optim.state_dict(), "schedule_steps": self.optim_schedule.n_current_steps,
              "epoch": epoch, "best_val_metric": float(self.best_val_metric),
              "epochs_no_improve": int(self.epochs_no_improve)}
        sampler = getattr(self.train_data, "sampler", None)
        if sampler is not None and hasattr(sampler, "state_dict"):
            ck["sampler"] = sampler.state_dict()
        return ck

    def save(self, epoch: int, file_path: str = "output/bert_trained.model", is_best: bool = False) -> str:
        """``<file_path>.ep<epoch>`` and, ``is_best``, ``<file_path>.best.pth`` (:524-552) — as
        state_dict checkpoints (+ optimizer, LR-schedule, early-stopping and sampler state)
        instead of the reference's pickled module: loadable with weights_only=True."""
        path = f"{file_path}.ep{epoch}"
        if self.rank == 0:
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
            ck = self._checkpoint(epoch)
            torch.save(ck, path)
            if is_best:
                self.best_model_path = f"{file_path}.best.pth"
                torch.save(ck, self.best_model_path)
                print(f"Best model saved: {self.best_model_path}", flush=True)
            print(f"EP:{epoch} Model Saved: {path}", flush=True)
        return path

    def load(self, path: str) -> int:
        """Resume (train_embedding_rag.py:155-191).  A checkpoint of this trainer restores the
        weights and the optimizer / schedule / early-stopping / sampler state; the reference's
        formats (a pickled BERTFoundationModel, a state_dict or {'state_dict': ...}, optional
        ``module.`` prefixes) restore the weights, read by ``model.checkpoint`` without
        executing any pickled class.

        Returns the checkpoint's epoch; ``self.loaded_own_checkpoint`` says whether the file was
        this trainer's own (``save``: weights + optimizer state + epoch) — a reference-format file
        carries no epoch the resume may trust (the reference starts at --resume_epoch whatever the
        file holds, train_embedding_rag.py:155-191)."""
        from ..model.checkpoint import load_state_dict_any
        if torch.serialization.get_unsafe_globals_in_checkpoint(path):
            ck = {"model": load_state_dict_any(path)}
        else:
            ck = torch.load(path, map_location="cpu", weights_only=True)
        self.loaded_own_checkpoint = isinstance(ck, dict) and "model" in ck and "optim" in ck and "epoch" in ck
        sd = ck["model"] if "model" in ck else ck.get("state_dict", ck)
        sd = {k[7:] if k.startswith("module.") else k: v for k, v in sd.items()}
        self.model.load_state_dict(sd)
        self.flat.sync_mirror()
        if "optim" in ck:
            self.optim.load_state_dict(ck["optim"])
            self.optim_schedule.n_current_steps = int(ck.get("schedule_steps", 0))
        if "best_val_metric" in ck:
            self.best_val_metric = float(ck["best_val_metric"])
            self.epochs_no_improve = int(ck.get("epochs_no_improve", 0))
        sampler = getattr(self.train_data, "sampler", None)
        if "sampler" in ck and sampler is not None and hasattr(sampler, "load_state_dict"):
            sampler.load_state_dict(ck["sampler"])
        return int(ck.get("epoch", 0))

    def should_stop_early(self, val_metrics: Dict, epoch: Optional[int] = None) -> bool:
        """Early stopping on the validation ALT-class haplotype F1, hap_f1[1] (:490-522) — the
        reference computes it from the epoch's TP/FP/FN whatever ``val_metric`` says."""
        if "hap_tp" in val_metrics:
            _, _, f1 = self.calculate_metrics(val_metrics["hap_tp"], val_metrics["hap_fp"], val_metrics["hap_fn"])
            current = f1[1].item()
        else:
            current = float(val_metrics["overall_f1"])
        if getattr(self, "world", 1) > 1:
            # one decision for all ranks (the metrics are already global; rank 0's value is
            # broadcast so no rank can leave the epoch loop alone on a rounding difference)
            t = torch.tensor([current], dtype=torch.float64)
            if dist.get_backend() != "gloo":
                t = t.to(self.device)
            dist.broadcast(t, 0)
            current = float(t.item())
        if current > self.best_val_metric + self.min_delta:
            self.best_val_metric, self.epochs_no_improve = current, 0
            if self.rank == 0:
                print(f"New best {self.val_metric}: {current:.4f}", flush=True)
            return False
        self.epochs_no_improve += 1
        if self.rank == 0:
            print(f"No improvement for {self.epochs_no_improve} epoch(s) (best: {self.best_val_metric:.4f}, "
                  f"current: {current:.4f})", flush=True)
        return self.epochs_no_improve >= self.patience
