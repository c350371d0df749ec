"""ContrastiveTrainer — drop-in for reference src/training/trainer.py.

Same constructor, loop, metrics, checkpoint format and config look-ups as the reference
(trainer.py:19-323), including its quirk of reading FLAT keys (`eval_every`, `save_every`,
`gradient_clip_val`, `best_metric`, `eval_classifier_every`) from whatever dict it is given:
scripts/train.py passes the full nested config, so in a Hydra run those look-ups miss and the
defaults apply (SURVEY finding 4).  Kept on purpose so results match the reference.

MI355X additions (all optional, no behaviour change for a single process):
  * data parallel: with torch.distributed initialised and world_size > 1 the flat gradient is
    all-reduced (RCCL; bucketed behind the backward with distributed.GradBucketer) and averaged
    inside the fused Adam (phoneme_contrast_amd.distributed); the DataLoader is expected to hand
    each rank its own shard (scripts/train.py: ShardedBatchSampler).
  * FusedAdam fast path: when the optimizer is a FusedAdam the all-reduced flat buffer is passed
    straight to its single-kernel step.
  * perf.json: per epoch the train steps' wall time, samples/s over all ranks
    and the step's algorithmic TFLOP/s and GB/s with their fractions of the MI355X roofs
    (phoneme_contrast_amd.costs), written next to metrics.json.
  * loaders with `set_epoch` (GpuContrastiveBatches) get the trainer's epoch before each pass.
"""
import json
import logging
import time
from collections import defaultdict
from pathlib import Path
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
from torch.utils.data import DataLoader

from . import distributed as ddp

try:  # progress bars are cosmetic; the reference uses tqdm
    from tqdm import tqdm
except Exception:  # pragma: no cover
    def tqdm(it, **kw):
        return it


class ContrastiveTrainer:
    """Trainer for contrastive learning (reference trainer.py:19-323)."""

    def __init__(self, model: nn.Module, train_loader: DataLoader, val_loader: Optional[DataLoader],
                 loss_fn: nn.Module, optimizer, scheduler, device: torch.device,
                 config: Dict[str, Any], output_dir: Path, logger: logging.Logger):
        self.model = model
        self.train_loader = train_loader
        self.val_loader = val_loader
        self.loss_fn = loss_fn
        self.optimizer = optimizer
        self.scheduler = scheduler
        self.device = device
        self.config = config
        self.output_dir = Path(output_dir)
        self.logger = logger
        self.checkpoint_dir = self.output_dir / "checkpoints"
        self.checkpoint_dir.mkdir(parents=True, exist_ok=True)
        self.current_epoch = 0
        self.global_step = 0
        self.best_val_loss = float("inf")
        self.metrics_history = defaultdict(list)
        self.rank, self.world_size = ddp.world()
        self.perf_history = []

    # ------------------------------------------------------------------ loop
    def train(self, num_epochs: int) -> None:
        self.logger.info(f"Starting training for {num_epochs} epochs")
        self.logger.info(f"Training samples: {len(self.train_loader.dataset)}")
        if self.val_loader:
            self.logger.info(f"Validation samples: {len(self.val_loader.dataset)}")
        for epoch in range(num_epochs):
            self.current_epoch = epoch
            train_metrics = self._train_epoch()
            val_metrics = {}
            if self.val_loader and (epoch + 1) % self.config.get("eval_every", 1) == 0:
                val_metrics = self._validate()
            if self.val_loader and (epoch + 1) % self.config.get("eval_classifier_every", 5) == 0:
                val_metrics.update(self._evaluate_classifier(epoch + 1))
            if self.scheduler:
                self.scheduler.step()
            self._log_metrics(train_metrics, val_metrics)
            if (epoch + 1) % self.config.get("save_every", 10) == 0:
                self._save_checkpoint("periodic")
            best_metric = self.config.get("best_metric", "loss")
            metric_for_best = val_metrics.get(best_metric, float("inf"))
            if best_metric == "loss":
                is_best = metric_for_best < self.best_val_loss
            else:
                is_best = metric_for_best > self.best_val_loss
            if is_best:
                self.best_val_loss = metric_for_best
                self._save_checkpoint("best")
                self.logger.info(f"New best model! {best_metric}: {metric_for_best:.4f}")
        self._save_checkpoint("final")
        self._save_metrics()

    def _train_epoch(self) -> Dict[str, float]:
        self.model.train()
        if hasattr(self.train_loader, "set_epoch"):
            self.train_loader.set_epoch(self.current_epoch)
        total_loss, num_batches = 0.0, 0
        pbar = tqdm(self.train_loader, desc=f"Epoch {self.current_epoch + 1}",
                    disable=self.rank != 0)
        step_s, samples, shape = 0.0, 0, None
        for batch in pbar:
            views, labels = self._prepare_batch(batch)
            t0 = time.perf_counter()  # the train step proper (views already built): fwd, loss, bwd, step
            embeddings = self._forward_pass(views)
            loss = self.loss_fn(embeddings, labels)
            self.optimizer.zero_grad()
            loss.backward()
            self._reduce_clip_step()
            total_loss += loss.item()  # synchronises: the step has finished
            step_s += time.perf_counter() - t0
            samples += views.shape[0]
            shape = tuple(views.shape)
            num_batches += 1
            self.global_step += 1
            if hasattr(pbar, "set_postfix"):
                pbar.set_postfix({"loss": loss.item()})
        self._record_perf(num_batches, samples, step_s, shape)
        if self.world_size > 1:
            # BatchNorm running statistics are per rank during the epoch (each rank's batches);
            # like DDP's broadcast_buffers, validation and checkpoints use rank 0's
            ddp.broadcast_buffers(self.model)
        return {"loss": total_loss / max(num_batches, 1), "lr": self.optimizer.param_groups[0]["lr"]}

    def _grad_scale(self) -> float:
        """1/world for the per-rank (DDP-equivalent) loss; 1 for a global-batch loss
        (GlobalSupervisedContrastiveLoss), whose ranks' gradients are shares of one gradient."""
        return 1.0 if getattr(self.loss_fn, "global_batch", False) else 1.0 / self.world_size

    def _reduce_clip_step(self):
        """(all-reduce) -> (clip) -> optimizer step, in the reference's order (trainer.py:143-152).

        FusedAdam over every model parameter: the gradients stay in the backward's flat buffer
        (zero-copy views); with world_size > 1 it is summed by RCCL (in buckets behind the
        backward when a GradBucketer is attached) and the 1/world average is folded into the
        Adam kernel; clipping scales the summed buffer by min(1, clip / (||avg|| + 1e-6)) on the
        device (torch.nn.utils.clip_grad_norm_'s rule, no host sync).  Any other optimizer: the
        averaged gradient is written back into p.grad and torch's own clip / step run."""
        from .optim import FusedAdam
        clip = self.config.get("gradient_clip_val")
        opt = self.optimizer
        bucketer = getattr(self.model, "_grad_bucketer", None)
        pending = bucketer is not None and bucketer.pending()
        if isinstance(opt, FusedAdam) and ddp.covers(opt, self.model):
            flats, scale = None, 1.0
            if pending:  # buckets already summed behind the backward
                flats = bucketer.finish([sum(p.numel() for p in g["params"]) for g in opt.param_groups])
            elif self.world_size > 1:
                flats = opt.flat_grad_views()
                for f in flats:
                    ddp.allreduce_flat(f)
            if self.world_size > 1:
                scale = self._grad_scale()
            if clip:
                if flats is None:
                    flats = opt.flat_grad_views()
                ddp.clip_flat_(flats, float(clip), scale)
            opt.step(flat_grads=flats, grad_scale=scale)
            return
        grads = [p.grad for p in self.model.parameters() if p.grad is not None]
        if pending or self.world_size > 1:  # generic path: leave the AVERAGED gradient in p.grad
            if pending:  # the bucketer already summed the backward's flat buffer: no second reduce
                flat = bucketer.finish()[0]
            else:
                flat = torch.cat([g.reshape(-1) for g in grads])
                ddp.allreduce_flat(flat)
            if self.world_size > 1:
                flat = flat * self._grad_scale()
            off = 0
            for g in grads:
                g.copy_(flat[off:off + g.numel()].view_as(g))
                off += g.numel()
        if clip:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), clip)
        opt.step()

    def _validate(self) -> Dict[str, float]:
        self.model.eval()
        total_loss, num_batches = 0.0, 0
        with torch.no_grad():
            for batch in tqdm(self.val_loader, desc="Validation", disable=self.rank != 0):
                views, labels = self._prepare_batch(batch)
                embeddings = self._forward_pass(views)
                total_loss += self.loss_fn(embeddings, labels).item()
                num_batches += 1
        return {"loss": total_loss / max(num_batches, 1)}

    def _prepare_batch(self, batch: Dict) -> Tuple[torch.Tensor, torch.Tensor]:
        """[b, V, C, H, W] views -> [b*V, C, H, W], labels repeated V times (trainer.py:186-199)."""
        views = batch["views"].to(self.device)
        labels = torch.as_tensor(batch["label"]).to(self.device)
        if views.dim() == 5:
            b, v = views.shape[:2]
            views = views.view(b * v, *views.shape[2:])
            labels = labels.repeat_interleave(v)
        return views, labels

    def _forward_pass(self, views: torch.Tensor) -> torch.Tensor:
        return self.model(views)

    # ------------------------------------------------------------------ bookkeeping
    def _log_metrics(self, train_metrics: Dict, val_metrics: Dict) -> None:
        for k, v in train_metrics.items():
            self.metrics_history[f"train_{k}"].append(v)
        for k, v in val_metrics.items():
            self.metrics_history[f"val_{k}"].append(v)
        s = f"Epoch {self.current_epoch + 1} | Train Loss: {train_metrics['loss']:.4f}"
        if "loss" in val_metrics:
            s += f" | Val Loss: {val_metrics['loss']:.4f}"
        if "linear_accuracy" in val_metrics:
            s += f" | Linear Acc: {val_metrics['linear_accuracy']:.3f}"
        if "rf_accuracy" in val_metrics:
            s += f" | RF Acc: {val_metrics['rf_accuracy']:.3f}"
        s += f" | LR: {train_metrics['lr']:.6f}"
        self.logger.info(s)

    def _save_checkpoint(self, tag: str) -> None:
        if self.rank != 0:
            return
        checkpoint = {
            "epoch": self.current_epoch,
            "global_step": self.global_step,
            "model_state_dict": self.model.state_dict(),
            "optimizer_state_dict": self.optimizer.state_dict(),
            "scheduler_state_dict": self.scheduler.state_dict() if self.scheduler else None,
            "best_val_loss": self.best_val_loss,
            "config": self.config,
        }
        path = self.checkpoint_dir / f"checkpoint_{tag}.pt"
        torch.save(checkpoint, path)
        self.logger.info(f"Saved checkpoint: {path}")

    def _save_metrics(self) -> None:
        if self.rank != 0:
            return
        with open(self.output_dir / "metrics.json", "w") as f:
            json.dump(self.metrics_history, f, indent=2)
        with open(self.output_dir / "perf.json", "w") as f:
            json.dump({"world_size": self.world_size, "epochs": self.perf_history}, f, indent=2)

    def _record_perf(self, steps: int, samples: int, seconds: float, shape) -> None:
        """One perf.json entry per epoch: this rank's train-step time, samples/s
        of all ranks (each rank runs the same number of equal-size steps), and the step's
        algorithmic rates against the MI355X roofs for the per-rank batch shape."""
        from .costs import HBM_PEAK_GBS, model_step_cost
        rec = {"epoch": self.current_epoch, "steps": steps, "samples_per_rank": samples,
               "step_seconds": round(seconds, 4)}
        if steps and seconds > 0:
            rec["ms_per_step"] = round(1000.0 * seconds / steps, 3)
            rec["samples_per_s"] = round(self.world_size * samples / seconds, 1)
            cost = model_step_cost(self.model, shape[0], shape[-2], shape[-1]) if shape and len(shape) == 4 else None
            if cost is not None:
                fl, by, peak, xfl = cost
                per = seconds / steps
                # schema 2: mfma_fraction on the algorithmic (direct-conv) FLOPs, as bench.py; the FLOPs the
                # step executes (Winograd kernels: 16 multiplies per 2x2 output tile) as executed_mfma_fraction
                rec.update({"schema": 2, "step_tflops": round(xfl / per / 1e12, 2),
                            "step_gbps": round(by / per / 1e9, 1),
                            "mfma_fraction": round(fl / per / (peak * 1e12), 4),
                            "executed_mfma_fraction": round(xfl / per / (peak * 1e12), 4),
                            "hbm_fraction": round(by / per / (HBM_PEAK_GBS * 1e9), 4),
                            "cost_model": "phoneme_contrast_amd/costs.py (SURVEY 8(d)); last batch shape "
                                          f"{list(shape)}"})
        self.perf_history.append(rec)

    def load_checkpoint(self, path: Path) -> None:
        # every entry is a tensor or a plain container, so the safe loader reads it (as
        # scripts/evaluate.py:271 does with torch's default weights_only=True)
        checkpoint = torch.load(path, map_location=self.device, weights_only=True)
        self.model.load_state_dict(checkpoint["model_state_dict"])
        self.optimizer.load_state_dict(checkpoint["optimizer_state_dict"])
        if self.scheduler and checkpoint["scheduler_state_dict"]:
            self.scheduler.load_state_dict(checkpoint["scheduler_state_dict"])
        self.current_epoch = checkpoint["epoch"]
        self.global_step = checkpoint["global_step"]
        self.best_val_loss = checkpoint["best_val_loss"]
        self.logger.info(f"Loaded checkpoint from epoch {self.current_epoch}")

    def _evaluate_classifier(self, epoch: int) -> Dict[str, float]:
        """Linear / random-forest probes on embeddings (trainer.py:272-323; sklearn, CPU)."""
        self.model.eval()
        all_emb, all_lab = [], []
        with torch.no_grad():
            for batch in self.val_loader:
                views, lab = self._prepare_batch(batch)
                all_emb.append(self.model(views).cpu())
                all_lab.extend(lab.cpu().tolist())
            for batch in self.train_loader:
                views, lab = self._prepare_batch(batch)
                if views.dim() == 5:
                    views = views[:, 0]
                all_emb.append(self.model(views).cpu())
                all_lab.extend(lab.cpu().tolist())
        embeddings = torch.cat(all_emb, dim=0).numpy()
        labels = np.array(all_lab)
        results = {}
        from sklearn.ensemble import RandomForestClassifier
        from sklearn.linear_model import LogisticRegression
        from sklearn.model_selection import cross_val_score
        try:
            results["linear_accuracy"] = cross_val_score(
                LogisticRegression(max_iter=1000, random_state=42), embeddings, labels, cv=5).mean()
        except (ValueError, RuntimeError) as e:
            self.logger.warning(f"Linear classifier failed: {e}")
        try:
            results["rf_accuracy"] = cross_val_score(
                RandomForestClassifier(n_estimators=100, random_state=42), embeddings, labels, cv=5).mean()
        except (ValueError, RuntimeError) as e:
            self.logger.warning(f"Random Forest classifier failed: {e}")
        return results
