from phoneme_contrast_amd.trainer import ContrastiveTrainer  # noqa: F401
