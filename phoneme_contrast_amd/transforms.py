"""Spectrogram augmentations — drop-in for reference src/datasets/transforms.py.

Same classes, constructor arguments, seeding and `build_augmentation_pipeline` config contract.
Each transform's random draws are made on the host with exactly the reference's calls
(`random.seed(seed); torch.manual_seed(seed)`, the `random.random() < prob` coin, then
torchaudio.functional.mask_along_axis's two `torch.rand(1)` draws for a mask band, or
`random.uniform` + `torch.randn_like` for the noise), so the bands and levels are identical to the
reference's for the same seed.  Applying them is one libpcx launch (`pcx_specaug`) for a whole
batch of views (`Compose.apply_batch`), or for one view (`__call__`, the reference's signature).

Noise: by default the N(0, 1) tensor comes from a counter-based generator on the GPU (same
distribution, not torch's CPU stream); `exact_noise=True` draws it on the host with
`torch.randn` after the reference's seeding (bit-identical, slower: 8040 draws per view).
"""
import ctypes
import random
from typing import List, Optional, Sequence

import torch

from . import _lib


def mask_band(size: int, mask_param: int):
    """torchaudio.functional.mask_along_axis's draw (p = 1.0, iid_masks=False): [start, end)."""
    if mask_param < 1:
        return None
    value = torch.rand(1) * mask_param
    min_value = torch.rand(1) * (size - value)
    start = int(min_value.long().item())
    end = int((min_value.long() + value.long()).item())
    return (start, end)


class BaseTransform:
    """Base class for augmentations (transforms.py:9-22)."""

    kind = None

    def draw(self, shape, seed: Optional[int]):
        raise NotImplementedError

    def __call__(self, x: torch.Tensor, seed: Optional[int] = None) -> torch.Tensor:
        return Compose([self])(x, seed=seed, _offsets=False)


class TimeMask(BaseTransform):
    """Randomly mask consecutive time steps (transforms.py:25-48; torchaudio TimeMasking)."""

    kind = "time"

    def __init__(self, max_width: int = 30, prob: float = 0.5):
        self.max_width = max_width
        self.prob = prob

    def draw(self, shape, seed):
        if seed is not None:
            seed = int(seed)
            random.seed(seed)
            torch.manual_seed(seed)
        if random.random() < self.prob:
            return mask_band(shape[-1], self.max_width)
        return None


class FrequencyMask(BaseTransform):
    """Randomly mask consecutive frequency bins (transforms.py:51-74; torchaudio FrequencyMasking)."""

    kind = "freq"

    def __init__(self, max_width: int = 10, prob: float = 0.5):
        self.max_width = max_width
        self.prob = prob

    def draw(self, shape, seed):
        if seed is not None:
            seed = int(seed)
            random.seed(seed)
            torch.manual_seed(seed)
        if random.random() < self.prob:
            return mask_band(shape[-2], self.max_width)
        return None


class GaussianNoise(BaseTransform):
    """x + randn * U(min_snr, max_snr) with probability prob (transforms.py:77-97)."""

    kind = "noise"

    def __init__(self, min_snr: float = 0.001, max_snr: float = 0.005, prob: float = 0.3,
                 exact_noise: bool = False):
        self.min_snr = min_snr
        self.max_snr = max_snr
        self.prob = prob
        self.exact_noise = exact_noise

    def draw(self, shape, seed):
        if seed is not None:
            seed = int(seed)
            random.seed(seed)
            torch.manual_seed(seed)
        if random.random() < self.prob:
            level = random.uniform(self.min_snr, self.max_snr)
            noise = torch.randn(tuple(shape)) if self.exact_noise else None
            return (level, noise)
        return None


class TimeStretch(BaseTransform):
    """The reference's TimeStretch draws a rate and returns its input unchanged (transforms.py:100-126)."""

    kind = "identity"

    def __init__(self, min_rate: float = 0.9, max_rate: float = 1.1, prob: float = 0.5):
        self.min_rate = min_rate
        self.max_rate = max_rate
        self.prob = prob

    def draw(self, shape, seed):
        if seed is not None:
            seed = int(seed)
            random.seed(seed)
            torch.manual_seed(seed)
        if random.random() < self.prob:
            random.uniform(self.min_rate, self.max_rate)
        return None


class Compose:
    """Sequential pipeline; transform i is seeded with seed + 1000 i (transforms.py:129-144)."""

    def __init__(self, transforms: list):
        self.transforms = transforms
        kinds = [t.kind for t in transforms if t.kind != "identity"]
        # the fused kernel applies time band, frequency band, then noise; the reference's builder
        # only ever produces that order (transforms.py:160-182)
        order = {"time": 0, "freq": 1, "noise": 2}
        if [order[k] for k in kinds] != sorted(order[k] for k in kinds) or len(set(kinds)) != len(kinds):
            raise ValueError(f"unsupported transform order for the fused kernel: {kinds}")

    def draw(self, shape, seed: Optional[int], _offsets: bool = True):
        """Per-view parameters {'time': band|None, 'freq': band|None, 'noise': (level, noise)|None}."""
        out = {"time": None, "freq": None, "noise": None}
        for i, t in enumerate(self.transforms):
            s = None if seed is None else (seed + i * 1000 if _offsets else seed)
            p = t.draw(shape, s)
            if t.kind in out:
                out[t.kind] = p
        return out

    def native_config(self):
        """pcx_aug_config for the native draws, or None when a transform needs the Python path
        (exact host noise, TimeStretch's extra draws)."""
        cfg = _lib.AugConfig()
        for t in self.transforms:
            if isinstance(t, TimeMask):
                cfg.time_enabled, cfg.time_width, cfg.time_prob = 1, int(t.max_width), float(t.prob)
            elif isinstance(t, FrequencyMask):
                cfg.freq_enabled, cfg.freq_width, cfg.freq_prob = 1, int(t.max_width), float(t.prob)
            elif isinstance(t, GaussianNoise) and not t.exact_noise:
                cfg.noise_enabled = 1
                cfg.noise_min, cfg.noise_max, cfg.noise_prob = float(t.min_snr), float(t.max_snr), float(t.prob)
            else:
                return None
        return cfg

    def draw_batch(self, seeds: Sequence[int], F_: int, T_: int):
        """(tband [n,2], fband [n,2], level [n]) int32/int32/float32 CPU tensors via libpcx's
        bit-exact C++ reproduction of the reference's draws (csrc/draws.hip)."""
        cfg = self.native_config()
        if cfg is None:
            raise ValueError("pipeline needs the Python draw path")
        n = len(seeds)
        sd = torch.tensor([int(s) for s in seeds], dtype=torch.int64)
        tb = torch.zeros(n, 2, dtype=torch.int32)
        fb = torch.zeros(n, 2, dtype=torch.int32)
        lv = torch.zeros(n, dtype=torch.float32)
        _lib.check(_lib.lib().pcx_draw_view_params(None, _lib.ptr(sd), n, F_, T_, ctypes.byref(cfg), None,
                                                   _lib.ptr(tb), _lib.ptr(fb), _lib.ptr(lv)), "pcx_draw_view_params")
        return tb, fb, lv

    def apply_batch(self, x: torch.Tensor, seeds: Sequence[Optional[int]], _offsets: bool = True) -> torch.Tensor:
        """In place on x [n, ..., F, T] (CUDA): view i augmented with seeds[i]."""
        _lib.require_gpu(x, what="Compose")
        if not x.is_contiguous() or x.dtype != torch.float32:
            raise ValueError("apply_batch needs a contiguous float32 tensor")
        n = x.shape[0]
        if len(seeds) != n:
            raise ValueError(f"{len(seeds)} seeds for {n} views")
        F_, T_ = x.shape[-2], x.shape[-1]
        if _offsets and n and all(s is not None for s in seeds) and self.native_config() is not None:
            # device copies held in locals until the launch is enqueued (a freed temporary's block
            # could be handed to the next copy before the kernel reads it)
            tb, fb, lv = (t.to(x.device) for t in self.draw_batch(seeds, F_, T_))
            _lib.check(_lib.lib().pcx_specaug(_lib.ptr(x), n, F_, T_, _lib.ptr(tb), _lib.ptr(fb), _lib.ptr(lv), None,
                                              int(seeds[0]) & ((1 << 64) - 1), _lib.stream_of(x)), "pcx_specaug")
            return x
        view_shape = (1,) * (x.dim() - 2) + (F_, T_)
        tb: List[int] = []
        fb: List[int] = []
        lv: List[float] = []
        noises = []
        any_t = any_f = any_n = False
        exact = False
        for s in seeds:
            p = self.draw(view_shape, s, _offsets)
            t, f, nz = p["time"], p["freq"], p["noise"]
            tb += list(t) if t else [0, 0]
            fb += list(f) if f else [0, 0]
            any_t |= t is not None
            any_f |= f is not None
            if nz is not None:
                any_n = True
                lv.append(float(nz[0]))
                if nz[1] is not None:
                    exact = True
                noises.append(nz[1])
            else:
                lv.append(0.0)
                noises.append(None)
        dev = x.device
        tband = torch.tensor(tb, dtype=torch.int32).to(dev) if any_t else None
        fband = torch.tensor(fb, dtype=torch.int32).to(dev) if any_f else None
        level = torch.tensor(lv, dtype=torch.float32).to(dev) if any_n else None
        noise = None
        if exact:
            noise = torch.zeros(n, F_, T_, dtype=torch.float32)
            for i, z in enumerate(noises):
                if z is not None:
                    noise[i] = z.reshape(F_, T_)
            noise = noise.to(dev)
        seed0 = int(seeds[0]) if len(seeds) and seeds[0] is not None else 0
        _lib.check(_lib.lib().pcx_specaug(_lib.ptr(x), n, F_, T_, _lib.ptr(tband), _lib.ptr(fband), _lib.ptr(level),
                                          _lib.ptr(noise), seed0 & ((1 << 64) - 1), _lib.stream_of(x)),
                   "pcx_specaug")
        return x

    def __call__(self, x: torch.Tensor, seed: Optional[int] = None, _offsets: bool = True) -> torch.Tensor:
        """Reference signature: one view (any leading dims of size 1), returns a new tensor."""
        y = x.contiguous().float().clone().reshape((1,) + tuple(x.shape[-2:]))
        self.apply_batch(y, [seed], _offsets)
        return y.reshape(x.shape)


def build_augmentation_pipeline(config: dict) -> Compose:
    """Same config keys and defaults as the reference (transforms.py:147-182)."""
    transforms = []
    if config.get("time_mask", {}).get("enabled", False):
        params = config["time_mask"]
        transforms.append(TimeMask(max_width=params.get("max_width", 30), prob=params.get("prob", 0.5)))
    if config.get("freq_mask", {}).get("enabled", False):
        params = config["freq_mask"]
        transforms.append(FrequencyMask(max_width=params.get("max_width", 10), prob=params.get("prob", 0.5)))
    if config.get("noise", {}).get("enabled", False):
        params = config["noise"]
        transforms.append(GaussianNoise(min_snr=params.get("min_snr", 0.001), max_snr=params.get("max_snr", 0.005),
                                        prob=params.get("prob", 0.3), exact_noise=params.get("exact_noise", False)))
    return Compose(transforms)
