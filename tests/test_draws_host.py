"""libpcx's C++ reproduction of the reference's augmentation draws (csrc/draws.hip) equals the
Python / torch calls the reference makes (dataset.py:147-172, transforms.py:25-144).  Host only:
the library is loaded, no kernel is launched."""
import random

import pytest
import torch

from phoneme_contrast_amd import transforms as A
from phoneme_contrast_amd import _lib
from phoneme_contrast_amd.features import draw_gain


def _native_gains(seeds):
    sd = torch.tensor(seeds, dtype=torch.int64)
    out = torch.empty(len(seeds), dtype=torch.float32)
    _lib.check(_lib.lib().pcx_draw_view_params(_lib.ptr(sd), None, len(seeds), 1, 1, None, _lib.ptr(out), None,
                                               None, None), "draw")
    return out.tolist()


def test_gain_draws_bit_exact():
    seeds = list(range(0, 3000)) + [10000 * i + v for i in (17, 4095, 99999, 429496) for v in range(2)]
    want = [float(torch.tensor(draw_gain(s), dtype=torch.float32)) for s in seeds]
    assert _native_gains(seeds) == want


@pytest.mark.parametrize("probs", [(0.5, 0.5, 0.3), (0.7, 0.2, 0.9), (1.0, 1.0, 1.0)])
def test_augmentation_draws_bit_exact(probs):
    pipe = A.build_augmentation_pipeline({"time_mask": {"enabled": True, "max_width": 30, "prob": probs[0]},
                                          "freq_mask": {"enabled": True, "max_width": 10, "prob": probs[1]},
                                          "noise": {"enabled": True, "min_snr": 0.001, "max_snr": 0.005,
                                                    "prob": probs[2]}})
    seeds = [i * 20000 + v for i in range(700) for v in range(2)] + [2 ** 40 + 3]
    tb, fb, lv = pipe.draw_batch(seeds, 40, 201)
    for k, s in enumerate(seeds):
        p = pipe.draw((1, 1, 40, 201), s)
        assert tuple(tb[k].tolist()) == (p["time"] or (0, 0)), s
        assert tuple(fb[k].tolist()) == (p["freq"] or (0, 0)), s
        want = float(torch.tensor(p["noise"][0], dtype=torch.float32)) if p["noise"] else 0.0
        assert float(lv[k]) == want, s


def test_subset_pipeline_seed_slots():
    # only the enabled transforms take seed slots: freq mask alone is seeded with seed + 0
    pipe = A.build_augmentation_pipeline({"freq_mask": {"enabled": True, "prob": 0.9}})
    seeds = list(range(500))
    tb, fb, lv = pipe.draw_batch(seeds, 40, 201)
    for k, s in enumerate(seeds):
        assert tuple(fb[k].tolist()) == (pipe.draw((1, 1, 40, 201), s)["freq"] or (0, 0))
    assert int(tb.abs().sum()) == 0 and float(lv.abs().sum()) == 0.0
