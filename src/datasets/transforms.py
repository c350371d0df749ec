from phoneme_contrast_amd.transforms import *  # noqa: F401,F403
