from phoneme_contrast_amd.features import *  # noqa: F401,F403
