"""Feature path, host side (no GPU): the float64 oracle pinned where a pinned implementation exists
here (torch.stft), the float32 torchaudio matrices, and the augmentation draws / config contract
(reference src/datasets/features.py, transforms.py, dataset.py:147-172)."""
import math

import numpy as np
import pytest
import torch

from oracle import np_features as nf
from phoneme_contrast_amd import features as F
from phoneme_contrast_amd import transforms as A


def test_power_spectrogram_matches_torch_stft():
    # torchaudio.functional.spectrogram is torch.stft(center=True, reflect, hann periodic) |.|^2
    g = torch.Generator().manual_seed(0)
    wave = torch.randn(2, 3200, generator=g, dtype=torch.float64)
    ref = torch.stft(wave, n_fft=400, hop_length=160, win_length=400,
                     window=torch.hann_window(400, dtype=torch.float64), center=True, pad_mode="reflect",
                     normalized=False, onesided=True, return_complex=True).abs() ** 2
    got = nf.power_spectrogram(wave.numpy(), 400, 160)
    assert got.shape == tuple(ref.shape) == (2, 201, 21)
    np.testing.assert_allclose(got, ref.numpy(), rtol=1e-10, atol=1e-9)


def test_float32_filterbank_and_dct_match_oracle():
    fb = F.melscale_fbanks(201, 0.0, 8000.0, 80, 16000)
    assert fb.dtype == torch.float32 and fb.shape == (201, 80)
    # float32 (torchaudio computes the bank in float32) vs float64: <= 1e-5 on weights <= 1
    np.testing.assert_allclose(fb.numpy(), nf.melscale_fbanks(201, 0.0, 8000.0, 80, 16000), atol=1e-5)
    dct = F.create_dct(40, 80)
    ref = nf.create_dct(40, 80)
    np.testing.assert_allclose(dct.numpy(), ref, atol=5e-6)
    # DCT-II ortho: orthonormal columns
    np.testing.assert_allclose(ref.T @ ref, np.eye(40), atol=1e-12)


def test_amplitude_to_db_packing_rule():
    x = np.abs(np.random.default_rng(1).normal(size=(3, 4, 5))) * np.array([1.0, 1e-6, 1e-12])[:, None, None]
    per_clip = np.stack([nf.amplitude_to_db(x[i:i + 1])[0] for i in range(3)])
    batched = nf.amplitude_to_db(x)
    # a 3-D call floors every clip at the batch max - 80 dB; per-clip calls floor each clip at its own
    assert np.all(batched >= batched.max() - 80.0 - 1e-9)
    for i in range(3):
        assert np.all(per_clip[i] >= per_clip[i].max() - 80.0 - 1e-9)
    assert not np.allclose(per_clip, batched)


def test_deltas_oracle_on_ramp():
    c = np.arange(10, dtype=np.float64)[None, None, :] * 2.0
    d = nf.compute_deltas(c)
    np.testing.assert_allclose(d[0, 0, 2:-2], 2.0)  # interior slope of a ramp
    assert d[0, 0, 0] == pytest.approx((1 * (2 - 0) + 2 * (4 - 0)) / 10.0)  # replicate padding


def test_mask_band_draw_is_torchaudio_sequence():
    torch.manual_seed(7)
    v = torch.rand(1) * 30
    mv = torch.rand(1) * (201 - v)
    expect = (int(mv.long()), int(mv.long() + v.long()))
    torch.manual_seed(7)
    assert A.mask_band(201, 30) == expect
    for s in range(50):
        torch.manual_seed(s)
        a, b = A.mask_band(40, 10)
        assert 0 <= a <= b <= 40 and b - a < 10


def test_compose_seed_offsets_and_determinism():
    pipe = A.build_augmentation_pipeline({"time_mask": {"enabled": True, "max_width": 30, "prob": 1.0},
                                          "freq_mask": {"enabled": True, "max_width": 10, "prob": 1.0},
                                          "noise": {"enabled": True, "prob": 1.0}})
    assert [type(t).__name__ for t in pipe.transforms] == ["TimeMask", "FrequencyMask", "GaussianNoise"]
    p1 = pipe.draw((1, 1, 40, 201), 12345)
    p2 = pipe.draw((1, 1, 40, 201), 12345)
    assert p1["time"] == p2["time"] and p1["freq"] == p2["freq"] and p1["noise"][0] == p2["noise"][0]
    # transform i sees seed + 1000 i (transforms.py:139-143)
    assert pipe.transforms[1].draw((1, 1, 40, 201), 12345 + 1000) == p1["freq"]
    assert 0.001 <= p1["noise"][0] <= 0.005
    none = A.build_augmentation_pipeline({})
    assert none.transforms == [] and none.draw((1, 1, 40, 201), 1) == {"time": None, "freq": None, "noise": None}


def test_compose_rejects_order_the_fused_kernel_cannot_apply():
    with pytest.raises(ValueError):
        A.Compose([A.GaussianNoise(), A.TimeMask()])


def test_gain_draw_matches_dataset_sequence():
    import random
    for seed in (0, 10001, 420000):
        random.seed(seed)
        g = random.uniform(0.8, 1.2) if random.random() < 0.5 else 1.0
        assert F.draw_gain(seed) == g


def test_feature_path_has_no_cpu_fallback():
    fx = F.MFCCExtractor()
    with pytest.raises(RuntimeError, match="no CPU path"):
        fx(torch.zeros(2, 32000))
    assert F.build_feature_extractor({"type": "mfcc", "mfcc_params": {"n_mfcc": 13}}).n_mfcc == 13
    with pytest.raises(ValueError, match="Unknown feature extractor type"):
        F.build_feature_extractor({"type": "wav2vec"})
