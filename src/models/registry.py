from phoneme_contrast_amd.models import ModelRegistry, model_registry  # noqa: F401
