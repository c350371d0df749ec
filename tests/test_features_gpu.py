"""On-GPU feature path (csrc/mfcc.hip) vs the float64 oracle (oracle/np_features.py).

The oracle restates torchaudio 2.7.0 (absent here); its STFT step is pinned against torch.stft in
test_features_host.py, the mel / dB / DCT steps are PARITY UNPINNED (no reference fixture holds
feature values).  Tolerances: MFCC / log-mel values are tens to hundreds of dB-scaled units; fp32
|DFT|^2 accumulation gives ~1e-6 relative error in power, i.e. ~1e-5 dB, so 2e-3 absolute + 1e-5
relative is the bar (measured maxima are printed)."""
import numpy as np
import pytest
import torch

from oracle import np_features as nf

pytestmark = pytest.mark.gpu


def _waves(n, S=32000, seed=0):
    g = torch.Generator().manual_seed(seed)
    # speech-like dynamics: a few loud segments over low noise, so the top_db floor binds
    w = 0.01 * torch.randn(n, S, generator=g)
    for i in range(n):
        a = int(torch.randint(0, S // 2, (1,), generator=g))
        w[i, a:a + S // 4] += torch.randn(S // 4, generator=g) * (0.5 + i)
    return w


def _close(got, ref, atol=2e-3, rtol=1e-5):
    err = np.abs(got - ref)
    print(f"max abs err {err.max():.3e} (max |ref| {np.abs(ref).max():.1f})")
    np.testing.assert_allclose(got, ref, atol=atol, rtol=rtol)


@pytest.mark.parametrize("S", [32000, 16123])
def test_mfcc_per_clip_floor(S):
    from phoneme_contrast_amd.features import MFCCExtractor
    w = _waves(3, S)
    fx = MFCCExtractor().cuda()
    got = fx(w.cuda(), clamp_group=1).cpu().numpy()
    ref = np.stack([nf.mfcc(w[i:i + 1].double().numpy())[0] for i in range(3)])[:, None]
    assert got.shape == (3, 1, 40, 1 + S // 160)
    _close(got, ref)


def test_mfcc_batched_call_keeps_torchaudio_packing():
    from phoneme_contrast_amd.features import MFCCExtractor
    w = _waves(4, seed=3)
    got = MFCCExtractor().cuda()(w.cuda()).cpu().numpy()  # [B, S] input: floor over the batch
    ref = nf.mfcc_extractor(w.double().numpy())
    _close(got, ref)


def test_mfcc_deltas_and_gain():
    from phoneme_contrast_amd.features import MFCCExtractor
    w = _waves(2, seed=5)
    gain = torch.tensor([0.83, 1.17])
    fx = MFCCExtractor(add_delta=True, add_delta_delta=True).cuda()
    got = fx(w.cuda(), gain=gain.cuda(), clamp_group=1).cpu().numpy()
    ref = np.concatenate([nf.mfcc_extractor((w[i:i + 1] * gain[i]).double().numpy(), add_delta=True,
                                            add_delta_delta=True) for i in range(2)])
    assert got.shape == (2, 1, 120, 201)
    _close(got, ref)
    only_dd = MFCCExtractor(add_delta_delta=True).cuda()(w.cuda(), gain=gain.cuda(), clamp_group=1).cpu().numpy()
    _close(only_dd, np.concatenate([ref[:, :, :40], ref[:, :, 80:]], axis=2))


def test_log_mel_extractor():
    from phoneme_contrast_amd.features import MelSpectrogramExtractor
    w = _waves(2, seed=9)
    got = MelSpectrogramExtractor().cuda()(w.cuda()).cpu().numpy()
    ref = nf.amplitude_to_db(nf.mel_spectrogram(w.double().numpy()), top_db=None)[:, None]
    _close(got, ref)


def test_specaug_bands_and_exact_noise():
    from phoneme_contrast_amd import transforms as A
    pipe = A.build_augmentation_pipeline({"time_mask": {"enabled": True, "prob": 0.7},
                                          "freq_mask": {"enabled": True, "prob": 0.7},
                                          "noise": {"enabled": True, "prob": 0.6, "exact_noise": True}})
    g = torch.Generator().manual_seed(11)
    x = torch.randn(16, 1, 40, 201, generator=g)
    seeds = [i * 20000 + v for i in range(8) for v in range(2)]
    y = pipe.apply_batch(x.clone().cuda(), seeds).cpu().numpy()
    for k, s in enumerate(seeds):
        p = pipe.draw((1, 1, 40, 201), s)
        noise = None
        if p["noise"] is not None:
            noise = (p["noise"][1] * p["noise"][0]).numpy().reshape(40, 201)
        ref = nf.apply_masks(x[k, 0].double().numpy(), p["time"], p["freq"], noise)
        np.testing.assert_allclose(y[k, 0], ref, atol=1e-6, rtol=0)


def test_view_builder_matches_per_item_path():
    from phoneme_contrast_amd import transforms as A
    from phoneme_contrast_amd.features import GpuViewBuilder, MFCCExtractor, draw_gain
    pipe = A.build_augmentation_pipeline({"time_mask": {"enabled": True}, "freq_mask": {"enabled": True}})
    w = _waves(3, seed=21)
    idx = [5, 17, 40]
    views = GpuViewBuilder(MFCCExtractor().cuda(), pipe, n_views=2)(w.cuda(), idx).cpu().numpy()
    assert views.shape == (3, 2, 1, 40, 201)
    for i, d in enumerate(idx):
        for v in range(2):
            feat = nf.mfcc((w[i:i + 1] * draw_gain(d * 10000 + v)).double().numpy())[0]
            p = pipe.draw((1, 1, 40, 201), d * 20000 + v)
            _close(views[i, v, 0], nf.apply_masks(feat, p["time"], p["freq"]))
