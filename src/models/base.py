from phoneme_contrast_amd.models import BaseModel  # noqa: F401
