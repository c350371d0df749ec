from phoneme_contrast_amd.utils import get_best_device  # noqa: F401
