from phoneme_contrast_amd.models import PhonemeNet, PhonemeNetDeep, SpatialAttention  # noqa: F401
