"""float64 numpy restatement of the reference's feature path (test oracle, not product).

The reference computes features with torchaudio 2.7.0 (`uv.lock` pins torchaudio==2.7.0), which
is not installed here, so this restates torchaudio's published definitions as the reference calls
them:

* `MFCCExtractor` (src/datasets/features.py:22-103) = torchaudio.transforms.MFCC(sample_rate,
  n_mfcc, melkwargs={n_fft, hop_length, n_mels, f_min, f_max}), i.e. MelSpectrogram (hann window,
  periodic; center=True with reflect padding; power 2; HTK mel scale, norm=None) ->
  AmplitudeToDB("power", top_db=80) -> DCT-II (norm "ortho") -> first n_mfcc coefficients;
  optional ComputeDeltas(win_length=5, mode="replicate") for delta / delta-delta.
* `MelSpectrogramExtractor` (features.py:106-150) = MelSpectrogram -> AmplitudeToDB() (top_db None).
* SpecAugment-style transforms (src/datasets/transforms.py:25-97): TimeMask / FrequencyMask via
  torchaudio.functional.mask_along_axis (one band per call, [start, start + width) set to 0),
  GaussianNoise (x + randn * level), Compose seeds transform i with seed + 1000 i (:129-144).

Pinning: the STFT step is torch.stft itself (torchaudio.functional.spectrogram calls it), so
tests/test_features_oracle.py pins `power_spectrogram` against torch.stft; the mel filterbank,
dB conversion and DCT are restated from torchaudio's formulas with no reference fixture to check
them against -- PARITY UNPINNED for those steps (no test of the reference checks feature values).

`amplitude_to_db` keeps torchaudio's packing rule: for a 3-D input [B, F, T] the top_db floor is
taken over the whole packed batch; the reference's data path calls the extractor on one clip at
a time ([1, samples], dataset.py:86-90), so its floor is per clip.
"""
import math

import numpy as np


def hann_window(n):
    """torch.hann_window(n) (periodic=True): 0.5 - 0.5 cos(2 pi k / n)."""
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * math.pi * k / n)


def power_spectrogram(wave, n_fft=400, hop=160):
    """|STFT|^2, center=True reflect padding, onesided: wave [..., S] -> [..., n_fft//2+1, frames]
    (torchaudio.functional.spectrogram with power=2.0, normalized=False)."""
    wave = np.asarray(wave, dtype=np.float64)
    pad = n_fft // 2
    padded = np.pad(wave, [(0, 0)] * (wave.ndim - 1) + [(pad, pad)], mode="reflect")
    frames = 1 + (padded.shape[-1] - n_fft) // hop
    idx = np.arange(frames)[:, None] * hop + np.arange(n_fft)[None, :]
    seg = padded[..., idx] * hann_window(n_fft)            # [..., frames, n_fft]
    spec = np.fft.rfft(seg, axis=-1)                        # [..., frames, n_freq]
    return np.swapaxes(np.abs(spec) ** 2, -1, -2)


def hz_to_mel(f):
    return 2595.0 * np.log10(1.0 + np.asarray(f, dtype=np.float64) / 700.0)


def mel_to_hz(m):
    return 700.0 * (10.0 ** (np.asarray(m, dtype=np.float64) / 2595.0) - 1.0)


def melscale_fbanks(n_freqs, f_min, f_max, n_mels, sample_rate):
    """torchaudio.functional.melscale_fbanks(..., norm=None, mel_scale="htk") -> [n_freqs, n_mels]."""
    all_freqs = np.linspace(0, sample_rate // 2, n_freqs)
    m_pts = np.linspace(hz_to_mel(f_min), hz_to_mel(f_max), n_mels + 2)
    f_pts = mel_to_hz(m_pts)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts[None, :] - all_freqs[:, None]
    down = -slopes[:, :-2] / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return np.maximum(0.0, np.minimum(down, up))


def create_dct(n_mfcc, n_mels):
    """torchaudio.functional.create_dct(n_mfcc, n_mels, norm="ortho") -> [n_mels, n_mfcc]."""
    n = np.arange(n_mels, dtype=np.float64)
    k = np.arange(n_mfcc, dtype=np.float64)[:, None]
    dct = np.cos(math.pi / n_mels * (n + 0.5) * k)
    dct[0] *= 1.0 / math.sqrt(2.0)
    dct *= math.sqrt(2.0 / n_mels)
    return dct.T


def amplitude_to_db(x, top_db=80.0, amin=1e-10, multiplier=10.0):
    """torchaudio.functional.amplitude_to_DB with ref 1.0 (db_multiplier 0); the floor
    max - top_db is taken per packed [channels, F, T] block: over the batch of a 3-D input."""
    x_db = multiplier * np.log10(np.maximum(x, amin))
    if top_db is not None:
        shape = x_db.shape
        packed = shape[-3] if x_db.ndim > 2 else 1
        v = x_db.reshape(-1, packed, shape[-2], shape[-1])
        v = np.maximum(v, v.max(axis=(-3, -2, -1), keepdims=True) - top_db)
        x_db = v.reshape(shape)
    return x_db


def mel_spectrogram(wave, sample_rate=16000, n_fft=400, hop=160, n_mels=80, f_min=0.0, f_max=None):
    spec = power_spectrogram(wave, n_fft, hop)
    fb = melscale_fbanks(n_fft // 2 + 1, f_min, f_max or sample_rate / 2, n_mels, sample_rate)
    return np.swapaxes(np.swapaxes(spec, -1, -2) @ fb, -1, -2)


def mfcc(wave, sample_rate=16000, n_mfcc=40, n_fft=400, hop=160, n_mels=80, f_min=0.0, f_max=None,
         top_db=80.0):
    """torchaudio.transforms.MFCC forward: wave [B, S] -> [B, n_mfcc, frames] (features.py:44-55,77)."""
    mel = mel_spectrogram(wave, sample_rate, n_fft, hop, n_mels, f_min, f_max)
    mel_db = amplitude_to_db(mel, top_db=top_db)
    return np.swapaxes(np.swapaxes(mel_db, -1, -2) @ create_dct(n_mfcc, n_mels), -1, -2)


def compute_deltas(spec, win_length=5):
    """torchaudio.functional.compute_deltas(mode="replicate"): sum_k k (c[t+k] - c[t-k]) / (2 sum k^2)."""
    n = (win_length - 1) // 2
    denom = n * (n + 1) * (2 * n + 1) / 3.0
    padded = np.concatenate([np.repeat(spec[..., :1], n, axis=-1), spec,
                             np.repeat(spec[..., -1:], n, axis=-1)], axis=-1)
    T = spec.shape[-1]
    out = np.zeros_like(spec, dtype=np.float64)
    for k in range(-n, n + 1):
        out += k * padded[..., n + k:n + k + T]
    return out / denom


def mfcc_extractor(wave, n_mfcc=40, add_delta=False, add_delta_delta=False, **kw):
    """MFCCExtractor.forward (features.py:62-103) on [B, S]: [B, 1, n_feat, frames]."""
    base = mfcc(wave, n_mfcc=n_mfcc, **kw)
    feats = [base]
    if add_delta:
        feats.append(compute_deltas(base))
    if add_delta_delta:
        d = feats[1] if add_delta else compute_deltas(base)
        feats.append(compute_deltas(d))
    return np.concatenate(feats, axis=1)[:, None]


def apply_masks(x, t_band=None, f_band=None, noise=None):
    """Compose(TimeMask, FrequencyMask, GaussianNoise) on one view [F, T] given the drawn bands
    ([start, end) or None) and the drawn noise tensor (already scaled by its level) or None."""
    y = np.array(x, dtype=np.float64, copy=True)
    if t_band is not None:
        y[..., :, t_band[0]:t_band[1]] = 0.0
    if f_band is not None:
        y[..., f_band[0]:f_band[1], :] = 0.0
    if noise is not None:
        y = y + noise
    return y
