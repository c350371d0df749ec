from phoneme_contrast_amd.utils import adjust_params_for_system  # noqa: F401
