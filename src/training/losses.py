from phoneme_contrast_amd.losses import NTXentLoss, SupervisedContrastiveLoss, _LOSSES, get_loss_fn  # noqa: F401
