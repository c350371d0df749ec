"""`src.datasets` drop-in: the sampler, the GPU feature extractors and the augmentation pipeline
(the reference's dataset.py file IO is not part of the GPU path)."""
from phoneme_contrast_amd.features import (FeatureExtractor, GpuViewBuilder, MelSpectrogramExtractor,  # noqa: F401
                                           MFCCExtractor, build_feature_extractor)
from phoneme_contrast_amd.samplers import ContrastiveBatchSampler  # noqa: F401
from phoneme_contrast_amd.transforms import (Compose, FrequencyMask, GaussianNoise, TimeMask,  # noqa: F401
                                             TimeStretch, build_augmentation_pipeline)
