"""Feature extraction on the GPU — drop-in for reference src/datasets/features.py.

Same class names, constructor arguments, input-shape handling and output layout as the
reference's `MFCCExtractor` (features.py:22-103), `MelSpectrogramExtractor` (:106-150) and
`build_feature_extractor` (:153-165), which wrap torchaudio 2.7.0's MFCC / MelSpectrogram /
AmplitudeToDB / ComputeDeltas.  The arithmetic runs in libpcx (csrc/mfcc.hip): framing, window,
|DFT|^2 and the mel projection as MFMA GEMMs, then dB + DCT.  The filterbank and DCT matrices are
built here in float32 with torchaudio's own formulas (melscale_fbanks, create_dct).

`GpuViewBuilder` replaces the per-item feature work of `PhonemeContrastiveDataset.__getitem__`
(dataset.py:64-111) for a whole batch: the random gain (`_augment_waveform`, :147-172) and the
augmentation draws are made on the host with the reference's RNG calls and seeds
(idx * 10000 + view, idx * 20000 + view), the features and masks are computed in two launches.
"""
import math
import random
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn as nn

from . import _lib


# ----------------------------------------------------------------------------- torchaudio matrices
def melscale_fbanks(n_freqs: int, f_min: float, f_max: float, n_mels: int, sample_rate: int) -> torch.Tensor:
    """torchaudio.functional.melscale_fbanks(norm=None, mel_scale="htk") in float32: [n_freqs, n_mels]."""
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_min = 2595.0 * math.log10(1.0 + (f_min / 700.0))
    m_max = 2595.0 * math.log10(1.0 + (f_max / 700.0))
    m_pts = torch.linspace(m_min, m_max, n_mels + 2)
    f_pts = 700.0 * (10.0 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    zero = torch.zeros(1)
    down_slopes = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up_slopes = slopes[:, 2:] / f_diff[1:]
    return torch.max(zero, torch.min(down_slopes, up_slopes))


def create_dct(n_mfcc: int, n_mels: int) -> torch.Tensor:
    """torchaudio.functional.create_dct(n_mfcc, n_mels, norm="ortho") in float32: [n_mels, n_mfcc]."""
    n = torch.arange(float(n_mels))
    k = torch.arange(float(n_mfcc)).unsqueeze(1)
    dct = torch.cos(math.pi / float(n_mels) * (n + 0.5) * k)
    dct[0] *= 1.0 / math.sqrt(2.0)
    dct *= math.sqrt(2.0 / float(n_mels))
    return dct.t()


def _padded_fb(fb: torch.Tensor) -> torch.Tensor:
    nf, nm = fb.shape
    out = torch.zeros(((nf + 31) // 32) * 32, ((nm + 31) // 32) * 32)
    out[:nf, :nm] = fb
    return out


def _as_batch(waveform: torch.Tensor) -> torch.Tensor:
    """[samples] -> [1, samples]; [batch, 1, samples] -> [batch, samples] (features.py:70-75)."""
    if waveform.dim() == 1:
        waveform = waveform.unsqueeze(0)
    elif waveform.dim() == 3:
        waveform = waveform.squeeze(1)
    return waveform


class FeatureExtractor(nn.Module):
    """Base class for feature extractors (features.py:9-19)."""

    def forward(self, waveform: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError


class _MelBase(FeatureExtractor):
    def __init__(self, sample_rate, n_fft, hop_length, n_mels, f_min, f_max):
        super().__init__()
        self.sample_rate = sample_rate
        self.n_fft = n_fft
        self.hop_length = hop_length
        self.n_mels = n_mels
        fb = melscale_fbanks(n_fft // 2 + 1, f_min, f_max or sample_rate / 2, n_mels, sample_rate)
        self.register_buffer("fb_padded", _padded_fb(fb), persistent=False)

    def frames(self, samples: int) -> int:
        return 1 + samples // self.hop_length

    def _mel(self, wave: torch.Tensor, gain: Optional[torch.Tensor]):
        """mel [n, n_mels, T] and per-32-frame maxima [n, ceil(T/32)]."""
        lib = _lib.lib()
        n, S = wave.shape
        T = self.frames(S)
        mel = torch.empty(n, self.n_mels, T, device=wave.device, dtype=torch.float32)
        tmax = torch.empty(n, (T + 31) // 32, device=wave.device, dtype=torch.float32)
        fb = self.fb_padded
        for c0 in range(0, n, 65535):  # the view index is the grid's y dimension
            c1 = min(n, c0 + 65535)
            g = gain[c0:c1] if gain is not None else None
            _lib.check(lib.pcx_melspec(_lib.ptr(wave[c0:c1]), c1 - c0, S, _lib.ptr(g), _lib.ptr(fb), self.n_fft,
                                       self.hop_length, self.n_mels, fb.shape[0], fb.shape[1],
                                       _lib.ptr(mel[c0:c1]), _lib.ptr(tmax[c0:c1]), _lib.stream_of(wave)),
                       "pcx_melspec")
        return mel, tmax

    def _prep(self, waveform, gain):
        wave = _as_batch(waveform)
        _lib.require_gpu(wave, gain, what=type(self).__name__)
        if self.fb_padded.device != wave.device:  # the filterbank / DCT buffers follow the input
            self.to(wave.device)
        wave = wave.contiguous().float()
        if gain is not None:
            gain = gain.reshape(-1).contiguous().float()
            if gain.shape[0] != wave.shape[0]:
                raise ValueError(f"gain has {gain.shape[0]} entries for {wave.shape[0]} clips")
        return wave, gain


class MFCCExtractor(_MelBase):
    """torchaudio MFCC (+ optional deltas) on the GPU (reference features.py:22-103).

    forward(waveform, gain=None, clamp_group=None): `gain` [batch] scales each clip first (the
    dataset's random gain); `clamp_group` is the number of consecutive clips sharing
    AmplitudeToDB's top_db floor -- None keeps torchaudio's rule for the call (the whole batch of a
    [batch, samples] input), 1 is per clip as in the reference's per-item data path.
    """

    def __init__(self, sample_rate: int = 16000, n_mfcc: int = 40, n_fft: int = 400, hop_length: int = 160,
                 n_mels: int = 80, f_min: float = 0.0, f_max: Optional[float] = None, add_delta: bool = False,
                 add_delta_delta: bool = False):
        super().__init__(sample_rate, n_fft, hop_length, n_mels, f_min, f_max)
        self.n_mfcc = n_mfcc
        self.add_delta = add_delta
        self.add_delta_delta = add_delta_delta
        self.top_db = 80.0
        self.register_buffer("dct_mat", create_dct(n_mfcc, n_mels).contiguous(), persistent=False)

    @property
    def n_features(self) -> int:
        return self.n_mfcc * (1 + int(self.add_delta) + int(self.add_delta_delta))

    def forward(self, waveform: torch.Tensor, gain: Optional[torch.Tensor] = None,
                clamp_group: Optional[int] = None) -> torch.Tensor:
        wave, gain = self._prep(waveform, gain)
        n, S = wave.shape
        T = self.frames(S)
        mel, tmax = self._mel(wave, gain)
        G = n if clamp_group is None else int(clamp_group)
        nf = self.n_features
        out = torch.empty(n, nf, T, device=wave.device, dtype=torch.float32)
        gmax = torch.empty((n + G - 1) // G, device=wave.device, dtype=torch.float32)
        lib = _lib.lib()
        st = _lib.stream_of(wave)
        _lib.check(lib.pcx_mel_finish(_lib.ptr(mel), _lib.ptr(tmax), n, T, self.n_mels, G, self.top_db,
                                      _lib.ptr(self.dct_mat), self.n_mfcc, _lib.ptr(gmax), _lib.ptr(out),
                                      nf * T, st), "pcx_mel_finish")
        if self.add_delta or self.add_delta_delta:
            # delta of the MFCC block; delta-delta of the delta (features.py:86-100)
            M = self.n_mfcc
            d = torch.empty(n, M, T, device=wave.device, dtype=torch.float32)
            _lib.check(lib.pcx_compute_deltas(_lib.ptr(out), nf * T, _lib.ptr(d), M * T, n, M, T, st),
                       "pcx_compute_deltas")
            k = 1
            if self.add_delta:
                out[:, M:2 * M] = d
                k = 2
            if self.add_delta_delta:
                dd = torch.empty_like(d)
                _lib.check(lib.pcx_compute_deltas(_lib.ptr(d), M * T, _lib.ptr(dd), M * T, n, M, T, st),
                           "pcx_compute_deltas")
                out[:, k * M:(k + 1) * M] = dd
        return out.unsqueeze(1)


class MelSpectrogramExtractor(_MelBase):
    """torchaudio MelSpectrogram -> AmplitudeToDB() (top_db None) on the GPU (features.py:106-150)."""

    def __init__(self, sample_rate: int = 16000, n_fft: int = 400, hop_length: int = 160, n_mels: int = 80,
                 f_min: float = 0.0, f_max: Optional[float] = None):
        super().__init__(sample_rate, n_fft, hop_length, n_mels, f_min, f_max)

    def forward(self, waveform: torch.Tensor, gain: Optional[torch.Tensor] = None) -> torch.Tensor:
        wave, gain = self._prep(waveform, gain)
        n, S = wave.shape
        T = self.frames(S)
        mel, tmax = self._mel(wave, gain)
        out = torch.empty(n, self.n_mels, T, device=wave.device, dtype=torch.float32)
        gmax = torch.empty(1, device=wave.device, dtype=torch.float32)
        _lib.check(_lib.lib().pcx_mel_finish(_lib.ptr(mel), _lib.ptr(tmax), n, T, self.n_mels, n, 0.0,
                                             _lib.ptr(None), self.n_mels, _lib.ptr(gmax), _lib.ptr(out),
                                             self.n_mels * T, _lib.stream_of(wave)), "pcx_mel_finish")
        return out.unsqueeze(1)


def build_feature_extractor(config: Dict) -> FeatureExtractor:
    """Same config contract as the reference (features.py:153-165)."""
    extractor_type = config.get("type", "mfcc")
    if extractor_type == "mfcc":
        return MFCCExtractor(**config.get("mfcc_params", {}))
    elif extractor_type == "mel":
        return MelSpectrogramExtractor(**config.get("mel_params", {}))
    raise ValueError(f"Unknown feature extractor type: {extractor_type}")


# ----------------------------------------------------------------------------- batched views
def draw_gain(seed: int) -> float:
    """PhonemeContrastiveDataset._augment_waveform's draw (dataset.py:147-172): same seeding calls,
    same order; returns the gain applied to the view (1.0 when the coin says no)."""
    seed = int(seed)
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if random.random() < 0.5:
        return random.uniform(0.8, 1.2)
    return 1.0


class GpuViewBuilder:
    """Batched replacement of the per-item view generation of PhonemeContrastiveDataset
    (dataset.py:64-111): views [N, V, 1, F, T] from fixed-length waveforms [N, S] on the GPU.

    indices: the dataset indices of the N clips (they seed the draws exactly as __getitem__ does).
    """

    def __init__(self, feature_extractor: MFCCExtractor, augmentation_pipeline=None, n_views: int = 2,
                 mode: str = "train"):
        self.fx = feature_extractor
        self.aug = augmentation_pipeline
        self.n_views = n_views if mode == "train" else 1
        self.mode = mode

    def __call__(self, waveforms: torch.Tensor, indices: Sequence[int]) -> torch.Tensor:
        _lib.require_gpu(waveforms, what="GpuViewBuilder")
        N, S = waveforms.shape[0], waveforms.shape[-1]
        V = self.n_views
        wave = waveforms.reshape(N, S).float()
        wave_v = wave.repeat_interleave(V, dim=0) if V > 1 else wave
        if self.mode == "train":  # bit-exact native reproduction of the per-view gain draws
            seeds = torch.tensor([int(idx) * 10000 + v for idx in indices for v in range(V)], dtype=torch.int64)
            gain_h = torch.empty(seeds.shape[0], dtype=torch.float32)
            _lib.check(_lib.lib().pcx_draw_view_params(_lib.ptr(seeds), None, seeds.shape[0], 1, 1, None,
                                                       _lib.ptr(gain_h), None, None, None), "pcx_draw_view_params")
        else:
            gain_h = torch.ones(N * V, dtype=torch.float32)
        gain_t = gain_h.to(wave.device)
        feats = self.fx(wave_v, gain=gain_t, clamp_group=1)  # [N*V, 1, F, T]: per-clip floor
        if self.mode == "train" and self.aug is not None:
            seeds = [int(idx) * 20000 + v for idx in indices for v in range(V)]
            self.aug.apply_batch(feats, seeds)
        F_, T_ = feats.shape[-2], feats.shape[-1]
        return feats.reshape(N, V, 1, F_, T_) if V > 1 else feats.reshape(N, 1, F_, T_)
