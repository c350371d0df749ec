from phoneme_contrast_amd.models import BaseModel, PhonemeNet, PhonemeNetDeep, model_registry  # noqa: F401

__all__ = ["BaseModel", "model_registry", "PhonemeNet", "PhonemeNetDeep"]
