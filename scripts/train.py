#!/usr/bin/env python
"""Training entry point — drop-in for the reference's scripts/train.py (Hydra CLI).

    python scripts/train.py [group=option] [key.path=value] [+new.key=value] ...
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 scripts/train.py ...

Same flow as the reference (scripts/train.py:24-200): compose the config, logger, seeds, device,
system adjustment, data, model from the registry, Adam (+ cosine schedule), loss from the loss
registry, ContrastiveTrainer.train.  Differences: the model / loss / optimizer step run in the
MI355X kernels (phoneme_contrast_amd), torchrun launches data-parallel training (one process
per GPU, gradients all-reduced over RCCL), and `accel.synthetic_data=true` trains on synthetic
MFCC views when the WAV dataset (and its torchaudio MFCC pipeline) is not available.
"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402
from torch.utils.data import DataLoader, Dataset, Sampler  # noqa: E402

from phoneme_contrast_amd import config as cfglib  # noqa: E402
from phoneme_contrast_amd import distributed as ddp  # noqa: E402
from phoneme_contrast_amd.losses import get_loss_fn  # noqa: E402
from phoneme_contrast_amd.models import model_registry  # noqa: E402
from phoneme_contrast_amd.optim import FusedAdam  # noqa: E402
from phoneme_contrast_amd.trainer import ContrastiveTrainer  # noqa: E402
from phoneme_contrast_amd.utils import adjust_params_for_system, create_logger, get_best_device  # noqa: E402


class SyntheticMFCCDataset(Dataset):
    """Random MFCC 'clips' with the reference dataset's item format: {'views': [V,1,40,T] (train) or
    [1,40,T] (val), 'label': int, 'index': int} (reference src/datasets/dataset.py:65-111)."""

    def __init__(self, n_items, n_classes, n_mfcc, n_frames, views, mode, seed):
        self.labels = [i % n_classes for i in range(n_items)]
        self.n_mfcc, self.n_frames, self.views, self.mode, self.seed = n_mfcc, n_frames, views, mode, seed

    def __len__(self):
        return len(self.labels)

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(self.seed * 100003 + idx)
        base = torch.randn(1, self.n_mfcc, self.n_frames, generator=g)
        if self.mode == "train":
            views = torch.stack([base + 0.1 * torch.randn(base.shape, generator=g) for _ in range(self.views)])
        else:
            views = base
        return {"views": views, "label": self.labels[idx], "index": idx}


class ClassBalancedBatchSampler(Sampler):
    """K classes x M samples per batch (views are added by the dataset), shuffled per epoch, each
    rank drawing its own batches (reference src/datasets/samplers.py:84-118 layout)."""

    def __init__(self, labels, classes_per_batch, samples_per_class, seed, rank=0, world=1):
        self.by_class = {}
        for i, l in enumerate(labels):
            self.by_class.setdefault(l, []).append(i)
        self.K, self.M, self.seed, self.rank, self.world = classes_per_batch, samples_per_class, seed, rank, world
        self.epoch = 0

    def __len__(self):
        return len(self.by_class) // self.K // self.world

    def __iter__(self):
        g = torch.Generator().manual_seed(self.seed + self.epoch)
        self.epoch += 1
        classes = list(self.by_class)
        order = torch.randperm(len(classes), generator=g).tolist()
        batches = []
        for s in range(0, len(order) - self.K + 1, self.K):
            idx = []
            for ci in order[s:s + self.K]:
                pool = self.by_class[classes[ci]]
                pick = torch.randint(0, len(pool), (self.M,), generator=g).tolist()
                idx += [pool[p] for p in pick]
            batches.append(idx)
        for b in batches[self.rank::self.world][:len(self)]:
            yield b


def setup_data(cfg, logger, rank, world):
    if not cfg.accel.get("synthetic_data", False):
        raise NotImplementedError(
            "WAV -> MFCC -> SpecAugment data path (reference src/datasets) is not part of this "
            "build yet (it needs torchaudio on the host; the on-GPU MFCC kernels are the next row "
            "of the plan).  Run with accel.synthetic_data=true.")
    s = cfg.accel.synthetic
    n_items = s.num_classes * s.samples_per_class
    n_mfcc = cfg.data.feature_extractor.mfcc_params.n_mfcc
    c = cfg.data.contrastive
    n_train = int(n_items * cfg.data.train_split)
    train = SyntheticMFCCDataset(n_train, s.num_classes, n_mfcc, s.n_frames, c.views_per_sample, "train",
                                 cfg.experiment.seed)
    val = SyntheticMFCCDataset(n_items - n_train, s.num_classes, n_mfcc, s.n_frames, 1, "val",
                               cfg.experiment.seed + 1)
    sampler = ClassBalancedBatchSampler(train.labels, c.classes_per_batch, c.samples_per_class,
                                        cfg.experiment.seed, rank, world)
    train_loader = DataLoader(train, batch_sampler=sampler, num_workers=0)
    val_loader = DataLoader(val, batch_size=cfg.training.batch_size, shuffle=False, num_workers=0)
    logger.info(f"Synthetic data: {len(train)} train / {len(val)} val clips, {s.num_classes} classes, "
                f"{len(sampler)} batches per epoch per rank")
    return train_loader, val_loader, s.num_classes


def setup_model(cfg, device):
    model = model_registry.create(cfg.model.type, dict(cfg.model)).to(device)
    ddp.broadcast_module(model)
    wd = cfg.training.get("weight_decay", 0)
    if cfg.accel.get("fused_adam", True):
        optimizer = FusedAdam(model.parameters(), lr=cfg.training.learning_rate, weight_decay=wd)
    else:
        optimizer = torch.optim.Adam(model.parameters(), lr=cfg.training.learning_rate, weight_decay=wd)
    scheduler = None
    if cfg.training.get("use_scheduler", False):
        scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(
            optimizer, T_max=cfg.training.epochs, eta_min=cfg.training.get("min_lr", 1e-6))
    loss_cfg = dict(cfg.training.loss)
    loss_fn = get_loss_fn(loss_cfg.pop("type"), **loss_cfg)
    return model, optimizer, scheduler, loss_fn


def main(cfg):
    rank, world, local = ddp.init_from_env()
    output_dir = Path(cfg.experiment.output_dir)
    logger = create_logger(output_dir / "logs", console_log_level=cfg.logging.level)
    if rank == 0:
        logger.info("Configuration:\n" + cfglib.to_yaml(cfg))
    torch.manual_seed(cfg.experiment.seed)
    torch.cuda.manual_seed_all(cfg.experiment.seed)
    device = get_best_device(cfg.get("device", "auto"), logger)
    cfg = adjust_params_for_system(cfg, device, logger)
    train_loader, val_loader, num_classes = setup_data(cfg, logger, rank, world)
    model, optimizer, scheduler, loss_fn = setup_model(cfg, device)
    trainer = ContrastiveTrainer(model=model, train_loader=train_loader, val_loader=val_loader,
                                 loss_fn=loss_fn, optimizer=optimizer, scheduler=scheduler,
                                 device=device, config=cfglib.to_container(cfg),
                                 output_dir=output_dir, logger=logger)
    trainer.train(num_epochs=cfg.training.epochs)
    logger.info("Training complete!")
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    overrides = [a for a in sys.argv[1:] if "=" in a]
    main(cfglib.compose(str(ROOT / "configs"), "config", overrides))
