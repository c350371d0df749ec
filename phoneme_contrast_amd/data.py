"""Training data path of scripts/train.py on the GPU — drop-in for the reference's
src/datasets/{parser,dataset}.py + DataLoader wiring (scripts/train.py:24-117).

The reference builds every view in DataLoader workers, one clip at a time on the CPU: load WAV ->
pad/trim -> random gain -> torchaudio MFCC -> SpecAugment (dataset.py:65-111).  Here the
waveforms of the split are loaded once and kept resident in HBM (`WaveformStore`: 2 s clips are
128 KB each), the reference's own `ContrastiveBatchSampler` picks the clip indices (bit-exact
batches), and `GpuViewBuilder` (features.py) builds a whole batch of views in two launches with
the reference's per-(index, view) seeds.  Batches come out as the reference's collated dicts
{'views': [b, V, 1, F, T], 'label': [b]} so ContrastiveTrainer._prepare_batch is unchanged.

Data parallel: `ShardedBatchSampler` hands rank r the batches r, r + world, ... of the global
sampler sequence (the same RNG stream on every rank), truncated to equal counts per rank, so every
class group of a batch stays on one rank (its SupCon positives are local) and world 1 reproduces
the reference's batch sequence exactly.
"""
import logging
import random
import re
import wave
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch.utils.data import Sampler

from .features import GpuViewBuilder


# ----------------------------------------------------------------------------- parser (parser.py)
def extract_phoneme_label(file_path: Path) -> str:
    """'da (short).wav' -> 'da', 'ada2.wav' -> 'ada' (reference src/datasets/parser.py:12-37)."""
    name = Path(file_path).stem.lower()
    name = re.sub(r"\s*\([^)]*\)", "", name)
    name = re.sub(r"\d+$", "", name)
    match = re.match(r"^([a-z]+)", name)
    if not match:
        raise ValueError(f"Cannot extract label from: {Path(file_path).name}")
    return match.group(1)


def extract_metadata(file_path: Path) -> Dict:
    """CV / VCV structure, gender, vowel context, short flag (parser.py:40-77)."""
    file_path = Path(file_path)
    parts = file_path.parts
    md = {"structure": "unknown", "gender": "unknown", "vowel_context": "unknown",
          "full_path": str(file_path), "filename": file_path.name}
    for i, part in enumerate(parts):
        if part.upper() in ("CV", "VCV"):
            md["structure"] = part.upper()
            if i + 1 < len(parts) and parts[i + 1].lower() in ("male", "female"):
                md["gender"] = parts[i + 1].lower()
            if part.upper() == "CV" and i + 2 < len(parts) and re.match(r"^_[aeiou]_$", parts[i + 2]):
                md["vowel_context"] = parts[i + 2]
    md["is_short"] = "short" in file_path.stem.lower()
    return md


def parse_dataset(data_dir: Path, logger: Optional[logging.Logger] = None
                  ) -> Tuple[List[Path], List[int], Dict[str, int], List[Dict]]:
    """rglob *.wav, labels from file names, sorted label map (parser.py:79-153)."""
    log = (lambda m, lv="info": getattr(logger, lv)(m)) if logger else (lambda m, lv="info": print(m))
    data_dir = Path(data_dir)
    if not data_dir.exists():
        raise FileNotFoundError(f"Data directory not found: {data_dir}")
    wav_files = list(data_dir.rglob("*.wav"))
    log(f"Found {len(wav_files)} .wav files")
    paths, labels, metas = [], [], []
    for f in wav_files:
        try:
            lab = extract_phoneme_label(f)
            md = extract_metadata(f)
            md["phoneme"] = lab
        except Exception as e:  # noqa: BLE001 - the reference skips any unparsable file
            log(f"Skipping file: {f.name} — {e}", "warning")
            continue
        paths.append(f)
        labels.append(lab)
        metas.append(md)
    uniq = sorted(set(labels))
    label_map = {lab: i for i, lab in enumerate(uniq)}
    log(f"Successfully parsed {len(paths)} files")
    log(f"Found {len(uniq)} unique phonemes: {uniq}")
    return paths, [label_map[lab] for lab in labels], label_map, metas


# ----------------------------------------------------------------------------- waveforms
def read_wav(path: Path) -> Tuple[np.ndarray, int]:
    """PCM WAV -> float32 [channels, samples] in [-1, 1) and the sample rate (torchaudio.load's
    normalisation for 8/16/24/32-bit integer PCM; 32-bit float WAV through scipy)."""
    try:
        with wave.open(str(path), "rb") as w:
            n, ch, sw, sr = w.getnframes(), w.getnchannels(), w.getsampwidth(), w.getframerate()
            raw = w.readframes(n)
        if sw == 1:
            x = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
        elif sw == 2:
            x = np.frombuffer(raw, "<i2").astype(np.float32) / 32768.0
        elif sw == 3:
            b = np.frombuffer(raw, np.uint8).reshape(-1, 3).astype(np.int32)
            v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
            x = (np.where(v >= 1 << 23, v - (1 << 24), v)).astype(np.float32) / float(1 << 23)
        else:
            x = np.frombuffer(raw, "<i4").astype(np.float32) / float(1 << 31)
        return x.reshape(-1, ch).T.copy(), sr
    except wave.Error:  # WAVE_FORMAT_IEEE_FLOAT and friends
        from scipy.io import wavfile
        sr, x = wavfile.read(str(path))
        x = x.astype(np.float32)
        return (x[None] if x.ndim == 1 else x.T).copy(), sr


def pad_or_trim(w: np.ndarray, max_samples: int, mode: str) -> np.ndarray:
    """Random crop / random left pad for training, centred for validation (dataset.py:174-203;
    the reference draws from Python's global `random`)."""
    length = w.shape[-1]
    if length > max_samples:
        start = random.randint(0, length - max_samples) if mode == "train" else (length - max_samples) // 2
        return w[..., start:start + max_samples]
    if length < max_samples:
        pad = max_samples - length
        left = random.randint(0, pad) if mode == "train" else pad // 2
        return np.pad(w, [(0, 0)] * (w.ndim - 1) + [(left, pad - left)])
    return w


class WaveformStore:
    """Fixed-length mono clips [N, S] resident on one device, with their integer labels."""

    def __init__(self, waves: torch.Tensor, labels: Sequence[int], metadata: Optional[List[Dict]] = None):
        if waves.dim() != 2:
            raise ValueError(f"waveforms must be [N, samples], got {tuple(waves.shape)}")
        self.waves = waves.contiguous().float()
        self.labels = [int(v) for v in labels]
        self.metadata = metadata or [{} for _ in self.labels]

    def __len__(self):
        return len(self.labels)

    @classmethod
    def from_files(cls, file_paths, labels, metadata, target_sr, max_samples, mode, device):
        """Load + mono + pad/trim once (dataset.py:113-145).  Resampling to target_sr uses
        scipy's polyphase filter (torchaudio's sinc resampler is not in this image: values of a
        resampled clip are not bit-exact with the reference's)."""
        out = np.zeros((len(file_paths), max_samples), np.float32)
        for i, f in enumerate(file_paths):
            x, sr = read_wav(f)
            if sr != target_sr:
                from math import gcd

                from scipy.signal import resample_poly
                g = gcd(int(sr), int(target_sr))
                x = resample_poly(x, target_sr // g, sr // g, axis=-1).astype(np.float32)
            if x.shape[0] > 1:
                x = x.mean(axis=0, keepdims=True)
            out[i] = pad_or_trim(x, max_samples, mode)[0]
        return cls(torch.from_numpy(out).to(device), labels, metadata)

    @classmethod
    def synthetic(cls, num_classes, samples_per_class, clip_samples, seed, device, sample_rate=16000):
        """Random 'phoneme' clips: each class a fixed mix of three harmonics under a class
        envelope, each clip that mix at a random gain plus white noise.  Generated on the device
        from a seeded generator, so every rank builds the same store."""
        g = torch.Generator(device=device).manual_seed(int(seed))
        n = num_classes * samples_per_class
        t = torch.arange(clip_samples, device=device, dtype=torch.float32) / sample_rate
        f0 = 80.0 + 3000.0 * torch.rand(num_classes, 3, generator=g, device=device)
        amp = torch.rand(num_classes, 3, generator=g, device=device)
        env = torch.sin(torch.pi * t / t[-1].clamp(min=1e-6)) ** 2
        labels = torch.arange(num_classes, device=device).repeat_interleave(samples_per_class)
        waves = torch.empty(n, clip_samples, device=device)
        for c0 in range(0, n, 1024):  # bounded temporaries
            c1 = min(n, c0 + 1024)
            lab = labels[c0:c1]
            ph = 2 * torch.pi * f0[lab][:, :, None] * t[None, None, :]
            w = (amp[lab][:, :, None] * torch.sin(ph)).sum(1) * env
            w *= 0.1 + 0.4 * torch.rand(c1 - c0, 1, generator=g, device=device)
            w += 0.01 * torch.randn(c1 - c0, clip_samples, generator=g, device=device)
            waves[c0:c1] = w
        return cls(waves, labels.tolist())

    def subset(self, indices: Sequence[int]) -> "WaveformStore":
        idx = torch.as_tensor(list(indices), dtype=torch.long, device=self.waves.device)
        return WaveformStore(self.waves.index_select(0, idx), [self.labels[i] for i in indices],
                             [self.metadata[i] for i in indices])


# ----------------------------------------------------------------------------- batching
class ShardedBatchSampler(Sampler[List[int]]):
    """Rank r of `world` takes the global batches r, r + world, ... (equal counts per rank)."""

    def __init__(self, batch_sampler, rank: int = 0, world: int = 1):
        self.batch_sampler, self.rank, self.world = batch_sampler, int(rank), int(world)
        if len(batch_sampler) < self.world:
            raise ValueError(f"{len(batch_sampler)} batches per epoch cannot feed {self.world} ranks: use more "
                             "classes (or fewer classes_per_batch) so that every rank gets at least one batch")

    def __getattr__(self, k):  # valid_classes, classes_per_batch, ... of the wrapped sampler
        if k == "batch_sampler":
            raise AttributeError(k)
        return getattr(self.batch_sampler, k)

    def __iter__(self):
        batches = list(self.batch_sampler)  # the whole sequence: same RNG calls on every rank
        n = len(batches) // self.world
        yield from batches[self.rank::self.world][:n]

    def __len__(self):
        return len(self.batch_sampler) // self.world


class _Sized:
    def __init__(self, n, labels):
        self._n, self.labels = n, labels

    def __len__(self):
        return self._n


class GpuContrastiveBatches:
    """The train loader: for every sampler batch (clip indices of the split) the views
    [b, V, 1, F, T] built on the GPU, as the reference's collated batch dict."""

    def __init__(self, store: WaveformStore, batch_sampler, builder: GpuViewBuilder):
        self.store, self.batch_sampler, self.builder = store, batch_sampler, builder
        self.dataset = _Sized(len(store), store.labels)

    def __len__(self):
        return len(self.batch_sampler)

    def __iter__(self):
        dev = self.store.waves.device
        for idx in self.batch_sampler:
            ix = torch.as_tensor([int(i) for i in idx], dtype=torch.long, device=dev)
            views = self.builder(self.store.waves.index_select(0, ix), [int(i) for i in idx])
            labels = torch.as_tensor([self.store.labels[int(i)] for i in idx], dtype=torch.long)
            yield {"views": views, "label": labels, "index": ix}


class GpuEvalBatches:
    """The validation loader: consecutive clips, one unaugmented view each ([b, 1, F, T])."""

    def __init__(self, store: WaveformStore, batch_size: int, builder: GpuViewBuilder):
        self.store, self.batch_size, self.builder = store, int(batch_size), builder
        self.dataset = _Sized(len(store), store.labels)

    def __len__(self):
        return (len(self.store) + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        for s in range(0, len(self.store), self.batch_size):
            idx = list(range(s, min(len(self.store), s + self.batch_size)))
            views = self.builder(self.store.waves[s:idx[-1] + 1], idx)
            labels = torch.as_tensor(self.store.labels[s:idx[-1] + 1], dtype=torch.long)
            yield {"views": views, "label": labels, "index": torch.as_tensor(idx)}
