"""Drop-in import surface: `src.models`, `src.training`, `src.utils` resolve to the MI355X-native
implementation in phoneme_contrast_amd, so the reference's scripts and tests import unchanged."""
