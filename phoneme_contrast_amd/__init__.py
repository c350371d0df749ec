"""phoneme_contrast_amd — MI355X-native (gfx950) contrastive phoneme train step.

Drop-in for the reference's `src.models` / `src.training` hot path: same registries, class names,
state_dict keys, loss semantics and trainer contract; the arithmetic runs in hand-written HIP
kernels (libpcx.so, C ABI in include/pcx.h).  See DESIGN.md.
"""
from .losses import NTXentLoss, SupervisedContrastiveLoss, get_loss_fn  # noqa: F401

__version__ = "0.1.0"
