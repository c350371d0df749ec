#!/usr/bin/env python
"""Training entry point — drop-in for the reference's scripts/train.py (Hydra CLI).

    python scripts/train.py [group=option] [key.path=value] [+new.key=value] ...
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 scripts/train.py ...

Same flow as the reference (scripts/train.py:24-200): compose the config, logger, seeds, device,
system adjustment, data, model from the registry, Adam (+ cosine schedule), loss from the loss
registry, ContrastiveTrainer.train.  Differences: the model / loss / optimizer step run in the
MI355X kernels (phoneme_contrast_amd); the data path keeps the clips in HBM and builds the
MFCC / SpecAugment views on the GPU (phoneme_contrast_amd.data) with the reference's sampler;
torchrun launches data-parallel training (one process per GPU, gradients all-reduced over RCCL
in buckets behind the backward); `accel.synthetic_data=true` trains on synthetic clips when the
WAV dataset is not available.  The per-rank batch is classes_per_batch x samples_per_class x
views_per_sample embeddings, e.g. the BASELINE's 4096 per GPU:

    python scripts/train.py accel.synthetic_data=true accel.synthetic.num_classes=20000 \
        data.contrastive.classes_per_batch=1024
"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402
from phoneme_contrast_amd import config as cfglib  # noqa: E402
from phoneme_contrast_amd import distributed as ddp  # noqa: E402
from phoneme_contrast_amd.data import (GpuContrastiveBatches, GpuEvalBatches, ShardedBatchSampler,  # noqa: E402
                                       WaveformStore, parse_dataset)
from phoneme_contrast_amd.features import GpuViewBuilder, build_feature_extractor  # noqa: E402
from phoneme_contrast_amd.losses import GlobalSupervisedContrastiveLoss, get_loss_fn  # noqa: E402
from phoneme_contrast_amd.models import model_registry  # noqa: E402
from phoneme_contrast_amd.optim import FusedAdam  # noqa: E402
from phoneme_contrast_amd.samplers import ContrastiveBatchSampler  # noqa: E402
from phoneme_contrast_amd.trainer import ContrastiveTrainer  # noqa: E402
from phoneme_contrast_amd.transforms import build_augmentation_pipeline  # noqa: E402
from phoneme_contrast_amd.utils import adjust_params_for_system, create_logger, get_best_device  # noqa: E402


def setup_data(cfg, logger, rank, world, device):
    """Reference scripts/train.py:24-117 on the GPU data path (phoneme_contrast_amd.data):
    parse the WAV tree (or build synthetic clips: accel.synthetic_data=true), the same seeded
    85/15 randperm split, waveforms resident in HBM, the reference's ContrastiveBatchSampler
    (sharded over ranks), views built on the GPU by GpuViewBuilder."""
    fx = build_feature_extractor(dict(cfg.data.feature_extractor))
    aug = build_augmentation_pipeline(dict(cfg.data.augmentation))
    target_sr = cfg.data.get("target_sr", 16000)
    max_samples = int(cfg.data.get("max_length_ms", 2000) * target_sr / 1000)
    if cfg.accel.get("synthetic_data", False):
        s = cfg.accel.synthetic
        store = WaveformStore.synthetic(s.num_classes, s.samples_per_class, s.get("clip_samples", max_samples),
                                        cfg.experiment.seed, device, target_sr)
        labels, n_classes = store.labels, s.num_classes
        logger.info(f"Synthetic data: {len(store)} clips of {store.max_samples} samples, {n_classes} classes")
    else:
        file_paths, labels, label_map, metadata = parse_dataset(Path(cfg.data.data_path), logger)
        store, n_classes = None, len(label_map)
    n_files = len(labels)
    n_train = int(n_files * cfg.data.train_split)
    indices = torch.randperm(n_files).tolist()  # the reference's split (seeded by experiment.seed)
    train_idx, val_idx = indices[:n_train], indices[n_train:]
    if store is not None:
        train_store, val_store = store.subset(train_idx), store.subset(val_idx)
        del store
    else:
        seed = cfg.experiment.seed  # crops drawn from (seed, epoch, clip): identical on every rank
        train_store = WaveformStore.from_files([file_paths[i] for i in train_idx], [labels[i] for i in train_idx],
                                               [metadata[i] for i in train_idx], target_sr, max_samples, "train",
                                               device, seed=seed)
        val_store = WaveformStore.from_files([file_paths[i] for i in val_idx], [labels[i] for i in val_idx],
                                             [metadata[i] for i in val_idx], target_sr, max_samples, "val", device,
                                             seed=seed)
    c = cfg.data.contrastive
    sampler = ContrastiveBatchSampler(labels=train_store.labels, classes_per_batch=c.classes_per_batch,
                                      samples_per_class=c.samples_per_class, views_per_sample=c.views_per_sample,
                                      shuffle=True, seed=cfg.experiment.seed, min_samples_to_exclude=0)
    logger.info(f"Total unique classes in training: {len(set(train_store.labels))}")
    logger.info(f"Classes in sampler: {len(sampler.valid_classes)}")
    logger.info(f"Classes per batch: {c.classes_per_batch}")
    logger.info(f"Samples per class: {c.samples_per_class}")
    logger.info(f"Total batches per epoch: {len(sampler)}")
    sharded = ShardedBatchSampler(sampler, rank, world)
    train_loader = GpuContrastiveBatches(train_store, sharded,
                                         GpuViewBuilder(fx, aug, c.views_per_sample, mode="train"))
    val_loader = GpuEvalBatches(val_store, cfg.training.batch_size, GpuViewBuilder(fx, None, 1, mode="val"))
    logger.info(f"Rank {rank}/{world}: {len(sharded)} batches per epoch of {c.classes_per_batch} classes x "
                f"{c.samples_per_class} samples x {c.views_per_sample} views = "
                f"{c.classes_per_batch * c.samples_per_class * c.views_per_sample} embeddings")
    return train_loader, val_loader, n_classes


def setup_model(cfg, device, world=1):
    model = model_registry.create(cfg.model.type, dict(cfg.model)).to(device)
    ddp.broadcast_module(model)
    wd = cfg.training.get("weight_decay", 0)
    if cfg.accel.get("fused_adam", True):
        optimizer = FusedAdam(model.parameters(), lr=cfg.training.learning_rate, weight_decay=wd)
    else:
        optimizer = torch.optim.Adam(model.parameters(), lr=cfg.training.learning_rate, weight_decay=wd)
    if ddp.is_distributed() and isinstance(optimizer, FusedAdam) and ddp.covers(optimizer, model):
        # gradient all-reduce in buckets behind the native backward, handed to the fused step;
        # torch.optim.Adam takes the trainer's flat all-reduce into p.grad instead
        ddp.GradBucketer(model, bucket_bytes=int(cfg.accel.get("bucket_mb", 4) * (1 << 20)))
    scheduler = None
    if cfg.training.get("use_scheduler", False):
        scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(
            optimizer, T_max=cfg.training.epochs, eta_min=cfg.training.get("min_lr", 1e-6))
    loss_cfg = dict(cfg.training.loss)
    loss_type = loss_cfg.pop("type")
    if cfg.accel.get("global_supcon", False) and world > 1:
        if loss_type != "supervised_contrastive":
            raise ValueError(f"accel.global_supcon needs the supervised_contrastive loss, not {loss_type}")
        loss_fn = GlobalSupervisedContrastiveLoss(**loss_cfg)
    else:
        loss_fn = get_loss_fn(loss_type, **loss_cfg)
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
    logger.info("Setting up data...")
    train_loader, val_loader, num_classes = setup_data(cfg, logger, rank, world, device)
    logger.info(f"Train batches: {len(train_loader)}, Val batches: {len(val_loader)}")
    logger.info(f"Number of phoneme classes: {num_classes}")
    logger.info("Setting up model...")
    model, optimizer, scheduler, loss_fn = setup_model(cfg, device, world)
    trainer = ContrastiveTrainer(model=model, train_loader=train_loader, val_loader=val_loader,
                                 loss_fn=loss_fn, optimizer=optimizer, scheduler=scheduler,
                                 device=device, config=cfglib.to_container(cfg),
                                 output_dir=output_dir, logger=logger)
    logger.info("Starting training...")
    trainer.train(num_epochs=cfg.training.epochs)
    logger.info("Training complete!")
    if ddp.is_distributed():  # also the world-1 group PCX_DIST_FORCE_INIT=1 creates
        torch.distributed.destroy_process_group()
    return trainer


def cli():
    """Hydra when it is installed (the reference's @hydra.main), else the compose shim."""
    try:
        import hydra
        from omegaconf import OmegaConf
    except ImportError:
        overrides = [a for a in sys.argv[1:] if "=" in a]
        return main(cfglib.compose(str(ROOT / "configs"), "config", overrides))

    @hydra.main(version_base=None, config_path="../configs", config_name="config")
    def _main(cfg):
        return main(cfglib.wrap(OmegaConf.to_container(cfg, resolve=True)))

    return _main()


if __name__ == "__main__":
    cli()
