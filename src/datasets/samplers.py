from phoneme_contrast_amd.samplers import *  # noqa: F401,F403
