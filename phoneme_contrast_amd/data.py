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
    count = lambda key, val: sum(1 for m in metas if m[key] == val)  # noqa: E731
    log(f"Structure: CV={count('structure', 'CV')}, VCV={count('structure', 'VCV')}")
    log(f"Gender: Male={count('gender', 'male')}, Female={count('gender', 'female')}")
    vowels = {}
    for m in metas:
        if m["structure"] == "CV" and m["vowel_context"] != "unknown":
            vowels[m["vowel_context"]] = vowels.get(m["vowel_context"], 0) + 1
    if vowels:
        log(f"CV vowel contexts: {vowels}")
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


def pad_or_trim(w: np.ndarray, max_samples: int, mode: str, rng: Optional[random.Random] = None) -> np.ndarray:
    """Random crop / random left pad for training, centred for validation (dataset.py:174-203;
    the reference draws from Python's global `random`, here from `rng` when given)."""
    rnd = rng if rng is not None else random
    length = w.shape[-1]
    if length > max_samples:
        start = rnd.randint(0, length - max_samples) if mode == "train" else (length - max_samples) // 2
        return w[..., start:start + max_samples]
    if length < max_samples:
        pad = max_samples - length
        left = rnd.randint(0, pad) if mode == "train" else pad // 2
        return np.pad(w, [(0, 0)] * (w.ndim - 1) + [(left, pad - left)])
    return w


def _mix64(x: np.ndarray) -> np.ndarray:
    """splitmix64 finaliser (uint64 -> uint64), vectorised."""
    x = x.astype(np.uint64)
    with np.errstate(over="ignore"):
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def crop_shifts(lengths: np.ndarray, max_samples: int, seed: int, epoch: int, indices: np.ndarray) -> np.ndarray:
    """Per-clip source shift of the train-mode random crop / left pad: output sample j of clip i
    reads source sample j + shift_i (crop: shift = start in [0, len - max]; pad: shift = -left with
    left in [0, max - len]), each drawn uniformly from a counter hash of (seed, epoch, clip index),
    so every rank and every run draws the same crops."""
    lengths = np.asarray(lengths, np.int64)
    span = np.abs(lengths - max_samples)
    key = _mix64(np.uint64((int(seed) * 0x9E3779B97F4A7C15 + int(epoch)) & ((1 << 64) - 1)))
    h = _mix64(key ^ (np.asarray(indices, np.uint64) * np.uint64(0xD1B54A32D192ED03)))
    draw = (h % (span.astype(np.uint64) + np.uint64(1))).astype(np.int64)
    return np.where(lengths > max_samples, draw, -draw)


class WaveformStore:
    """Mono clips resident on one device, with their integer labels.

    Either fixed-length clips `waves` [N, S] (synthetic stores, validation, small train sets), or
    for a train set of >= 500 files the uncropped clips stored ragged -- one concatenated 1-D buffer
    `flat` with per-clip `offsets` / `lengths` (host arrays), so one long outlier clip costs its own
    length, not N times it: the reference reloads and re-crops such a set on every __getitem__
    (dataset.py:57-59,113-145), so `clips(indices, epoch)` draws a fresh crop / left pad per clip
    and epoch on the device (crop_shifts) and gathers it as flat[offset + j + shift].  Below 500
    files the reference caches the first crop, and so does this store (drawn once, at load)."""

    def __init__(self, waves: Optional[torch.Tensor], labels: Sequence[int], metadata: Optional[List[Dict]] = None,
                 flat: Optional[torch.Tensor] = None, lengths: Optional[Sequence[int]] = None,
                 max_samples: Optional[int] = None, seed: int = 0):
        if flat is None:
            if waves is None or waves.dim() != 2:
                raise ValueError(f"waveforms must be [N, samples], got {None if waves is None else tuple(waves.shape)}")
            self.waves = waves.contiguous().float()
            self.max_samples = self.waves.shape[1]
        else:
            self.waves = None
            self.flat = flat.contiguous().float().reshape(-1)
            self.lengths = np.asarray(lengths, np.int64)
            self.offsets = np.concatenate([[0], np.cumsum(self.lengths)[:-1]]).astype(np.int64)
            if int(self.lengths.sum()) != self.flat.numel():
                raise ValueError(f"ragged store: {self.flat.numel()} samples for clip lengths summing to "
                                 f"{int(self.lengths.sum())}")
            self.max_samples = int(max_samples)
            self.seed = int(seed)
        self.labels = [int(v) for v in labels]
        self.metadata = metadata or [{} for _ in self.labels]

    def __len__(self):
        return len(self.labels)

    @property
    def recrops(self) -> bool:
        return self.waves is None

    @property
    def device(self) -> torch.device:
        return (self.waves if self.waves is not None else self.flat).device

    def clips(self, indices, epoch: int = 0) -> torch.Tensor:
        """[n, max_samples] clips of `indices` for this epoch.  `indices` is a host sequence of
        clip numbers (the loaders pass the sampler's list: no device round trip) or a LongTensor."""
        if torch.is_tensor(indices):
            idx_np = indices.detach().cpu().numpy().astype(np.int64)
        else:
            idx_np = np.asarray(indices, np.int64).reshape(-1)
        dev = self.device
        if self.waves is not None:
            return self.waves.index_select(0, torch.as_tensor(idx_np, device=dev))
        ln_np = self.lengths[idx_np]
        shift = torch.as_tensor(crop_shifts(ln_np, self.max_samples, self.seed, epoch, idx_np), device=dev)
        ln = torch.as_tensor(ln_np, device=dev)
        base = torch.as_tensor(self.offsets[idx_np], device=dev)
        src = torch.arange(self.max_samples, device=dev)[None, :] + shift[:, None]
        valid = (src >= 0) & (src < ln[:, None])
        if self.flat.numel() == 0:
            return torch.zeros(len(idx_np), self.max_samples, device=dev)
        gidx = (base[:, None] + torch.minimum(src.clamp(min=0), (ln[:, None] - 1).clamp(min=0)))
        out = self.flat[gidx.clamp(0, self.flat.numel() - 1)]
        return out * valid

    @staticmethod
    def _load_mono(path, target_sr) -> np.ndarray:
        """Load + resample + mono (dataset.py:126-136) -> float32 [samples].  Resampling uses
        scipy's polyphase filter (torchaudio's sinc resampler is not in this image: values of a
        resampled clip are not bit-exact with the reference's)."""
        x, sr = read_wav(path)
        if sr != target_sr:
            from math import gcd

            from scipy.signal import resample_poly
            g = gcd(int(sr), int(target_sr))
            x = resample_poly(x, target_sr // g, sr // g, axis=-1).astype(np.float32)
        if x.shape[0] > 1:
            x = x.mean(axis=0, keepdims=True)
        return x[0]

    @classmethod
    def from_files(cls, file_paths, labels, metadata, target_sr, max_samples, mode, device, seed=0):
        """Load every clip of the split once (dataset.py:113-145).  Validation: centred crop / pad
        (deterministic).  Train with < 500 files: one seeded random crop / pad per clip, kept (the
        reference's cached path).  Train with >= 500 files: the uncropped clips stay in HBM and
        every epoch draws new crops (`clips`)."""
        mono = [cls._load_mono(f, target_sr) for f in file_paths]
        if mode == "train" and len(mono) >= 500:
            flat = np.concatenate(mono).astype(np.float32) if mono else np.zeros(0, np.float32)
            return cls(None, labels, metadata, flat=torch.from_numpy(flat).to(device),
                       lengths=[len(m) for m in mono], max_samples=max_samples, seed=seed)
        rng = random.Random(int(seed))
        out = np.zeros((len(mono), max_samples), np.float32)
        for i, m in enumerate(mono):
            out[i] = pad_or_trim(m[None], max_samples, mode, rng)[0]
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
        indices = list(indices)
        labels, meta = [self.labels[i] for i in indices], [self.metadata[i] for i in indices]
        if self.waves is not None:
            idx = torch.as_tensor(indices, dtype=torch.long, device=self.waves.device)
            return WaveformStore(self.waves.index_select(0, idx), labels, meta)
        parts = [self.flat[int(self.offsets[i]):int(self.offsets[i] + self.lengths[i])] for i in indices]
        flat = torch.cat(parts) if parts else self.flat[:0]
        return WaveformStore(None, labels, meta, flat=flat, lengths=self.lengths[np.asarray(indices, np.int64)],
                             max_samples=self.max_samples, seed=self.seed)


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
        self.epoch = 0  # crop epoch of the next pass (set_epoch; advances by itself as a fallback)

    def set_epoch(self, epoch: int) -> None:
        """Crop schedule of the next pass = (seed, epoch, clip), as DistributedSampler.set_epoch:
        ContrastiveTrainer._train_epoch calls it with its current_epoch, so an extra pass (warm-up,
        debug iteration) or a resumed run does not shift the crops."""
        self.epoch = int(epoch)

    def __len__(self):
        return len(self.batch_sampler)

    def __iter__(self):
        store = self.store
        dev = store.device
        epoch = self.epoch
        self.epoch += 1
        for idx in self.batch_sampler:
            idx = [int(i) for i in idx]
            views = self.builder(store.clips(idx, epoch), idx)
            labels = torch.as_tensor([self.store.labels[i] for i in idx], dtype=torch.long)
            yield {"views": views, "label": labels, "index": torch.as_tensor(idx, dtype=torch.long)}


class GpuEvalBatches:
    """The validation loader: consecutive clips, one unaugmented view each ([b, 1, F, T])."""

    def __init__(self, store: WaveformStore, batch_size: int, builder: GpuViewBuilder):
        self.store, self.batch_size, self.builder = store, int(batch_size), builder
        self.dataset = _Sized(len(store), store.labels)

    def __len__(self):
        return (len(self.store) + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        store = self.store
        for s in range(0, len(store), self.batch_size):
            idx = list(range(s, min(len(store), s + self.batch_size)))
            views = self.builder(store.clips(idx, 0), idx)
            labels = torch.as_tensor(self.store.labels[s:idx[-1] + 1], dtype=torch.long)
            yield {"views": views, "label": labels, "index": torch.as_tensor(idx)}
