"""ContrastiveBatchSampler — drop-in for reference src/datasets/samplers.py:11-118.

Same constructor, class filtering / oversampling rules, log lines and numpy RandomState call
sequence (shuffle of the class list, then one `choice` per class, with replacement only for
classes smaller than samples_per_class), so the batches are identical index for index
(tests/test_sampler.py against fixtures generated from the reference itself).  Host-side: the
indices it yields feed `GpuViewBuilder` (features.py), which builds the K x M x V views on the GPU.
"""
from collections import defaultdict
from typing import Iterator, List

import numpy as np
from torch.utils.data import Sampler

from .utils import get_logger


class ContrastiveBatchSampler(Sampler[List[int]]):
    """Batches of K classes x M samples per class (each sample later gives V views)."""

    def __init__(self, labels: List[int], classes_per_batch: int, samples_per_class: int,
                 views_per_sample: int, shuffle: bool = True, seed: int = 42,
                 min_samples_to_exclude: int = 0):
        self.labels = np.array(labels)
        self.classes_per_batch = classes_per_batch
        self.samples_per_class = samples_per_class
        self.views_per_sample = views_per_sample
        self.shuffle = shuffle
        self.seed = seed
        self.min_samples_to_exclude = min_samples_to_exclude

        self.label_to_indices = defaultdict(list)
        for idx, label in enumerate(labels):
            self.label_to_indices[label].append(idx)

        class_counts = {label: len(ix) for label, ix in self.label_to_indices.items()}
        logger = get_logger()
        logger.info(f"Class distribution: min={min(class_counts.values())}, max={max(class_counts.values())}")
        if min_samples_to_exclude > 0:
            self.valid_classes = [label for label, ix in self.label_to_indices.items()
                                  if len(ix) >= min_samples_to_exclude]
            excluded = set(self.label_to_indices.keys()) - set(self.valid_classes)
            if excluded:
                logger.warning(f"Excluded classes {sorted(excluded)} with < {min_samples_to_exclude} samples")
        else:
            self.valid_classes = list(self.label_to_indices.keys())
            under = [(label, len(ix)) for label, ix in self.label_to_indices.items() if len(ix) < samples_per_class]
            if under:
                logger.info("Classes requiring oversampling (sampling with replacement):")
                for label, count in sorted(under):
                    logger.info(f"  Class {label}: {count} samples (need {samples_per_class})")
        logger.info(f"Using {len(self.valid_classes)} classes for training")
        self.rng = np.random.RandomState(seed)

    def __iter__(self) -> Iterator[List[int]]:
        classes = self.valid_classes.copy()
        if self.shuffle:
            self.rng.shuffle(classes)
        for i in range(0, len(classes), self.classes_per_batch):
            batch_classes = classes[i:i + self.classes_per_batch]
            if len(batch_classes) < self.classes_per_batch:
                continue  # incomplete class groups are skipped
            batch = []
            for label in batch_classes:
                ix = self.label_to_indices[label]
                replace = len(ix) < self.samples_per_class
                batch.extend(self.rng.choice(ix, size=self.samples_per_class, replace=replace))
            yield batch

    def __len__(self) -> int:
        return len(self.valid_classes) // self.classes_per_batch
