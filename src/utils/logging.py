from phoneme_contrast_amd.utils import create_logger, get_logger  # noqa: F401
