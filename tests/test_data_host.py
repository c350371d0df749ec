"""The entry's real-data branch on the host (no GPU): WAV parsing and loading as
scripts/train.py:setup_data runs it (phoneme_contrast_amd.data).

* Every case of the reference's own parser tests (/root/reference/tests/test_parser.py:12-71 label
  regex, invalid names, CV / VCV metadata; :110-113 the missing-directory FileNotFoundError) against
  phoneme_contrast_amd.data.
* A temporary CV / VCV tree of `wave` files (16-bit mono 16 kHz, 16-bit stereo 22.05 kHz, 8-bit,
  24-bit, clips shorter and longer than 2 s): labels, the sorted label_map, read_wav's integer-PCM
  normalisation (torchaudio.load's x / 2^(bits-1)), mono mixdown, and the reference's pad / trim
  (src/datasets/dataset.py:174-203: centred for validation, random crop / left pad in range for
  training) through WaveformStore.from_files.
* The >= 500-file train store re-crops per epoch (dataset.py:57-59: no cache at that size), with
  draws that depend only on (seed, epoch, clip).
Resampled values are not compared bit-for-bit with torchaudio's sinc resampler (absent here):
parity unpinned for resampled clips; the resampled length and band-limited content are checked.
"""
import logging
import wave
from pathlib import Path

import numpy as np
import pytest
import torch

from phoneme_contrast_amd.data import (WaveformStore, crop_shifts, extract_metadata, extract_phoneme_label,
                                       pad_or_trim, parse_dataset, read_wav)


# ------------------------------------------------------------------ reference tests/test_parser.py
@pytest.mark.parametrize("filename,expected", [
    ("da.wav", "da"), ("da (short).wav", "da"), ("da1.wav", "da"), ("da1 (short).wav", "da"),
    ("ada2.wav", "ada"), ("bi (short version).wav", "bi"), ("apa.wav", "apa"),
])
def test_extract_phoneme_label(filename, expected):
    assert extract_phoneme_label(Path(filename)) == expected


def test_extract_phoneme_label_invalid():
    with pytest.raises(ValueError):
        extract_phoneme_label(Path("123.wav"))
    with pytest.raises(ValueError):
        extract_phoneme_label(Path("(short).wav"))


@pytest.mark.parametrize("path_str,expected", [
    ("data/raw/New Stimuli 9-8-2024/CV/Male/_a_/da.wav",
     {"structure": "CV", "gender": "male", "vowel_context": "_a_", "is_short": False}),
    ("data/raw/New Stimuli 9-8-2024/CV/Female/_i_/bi (short version).wav",
     {"structure": "CV", "gender": "female", "vowel_context": "_i_", "is_short": True}),
    ("data/raw/New Stimuli 9-8-2024/VCV/Female/ada2.wav",
     {"structure": "VCV", "gender": "female", "vowel_context": "unknown", "is_short": False}),
])
def test_extract_metadata(path_str, expected):
    md = extract_metadata(Path(path_str))
    for k, v in expected.items():
        assert md[k] == v
    assert md["filename"] == Path(path_str).name and md["full_path"] == str(Path(path_str))


def test_parse_dataset_missing_dir():
    with pytest.raises(FileNotFoundError):
        parse_dataset(Path("nonexistent/directory"))


# ------------------------------------------------------------------ a WAV tree
def _write(path: Path, data: np.ndarray, sr: int, width: int):
    """data: float [channels, n] in [-1, 1) -> integer PCM of `width` bytes."""
    path.parent.mkdir(parents=True, exist_ok=True)
    ch, n = data.shape
    inter = data.T.reshape(-1)
    if width == 1:
        raw = np.clip(np.round(inter * 128 + 128), 0, 255).astype(np.uint8).tobytes()
    elif width == 2:
        raw = np.clip(np.round(inter * 32768), -32768, 32767).astype("<i2").tobytes()
    else:  # 24-bit little endian
        v = np.clip(np.round(inter * (1 << 23)), -(1 << 23), (1 << 23) - 1).astype(np.int32)
        b = v.astype("<i4").view(np.uint8).reshape(-1, 4)[:, :3]
        raw = b.tobytes()
    with wave.open(str(path), "wb") as w:
        w.setnchannels(ch)
        w.setsampwidth(width)
        w.setframerate(sr)
        w.writeframes(raw)


# (relative path, channels, sample rate, bytes per sample, seconds)
TREE = [
    ("CV/Male/_a_/da.wav", 1, 16000, 2, 1.5),
    ("CV/Male/_a_/da1 (short).wav", 1, 16000, 2, 0.75),
    ("CV/Female/_i_/bi (short version).wav", 2, 22050, 2, 2.5),
    ("CV/Female/_e_/ga.wav", 1, 16000, 1, 2.0),
    ("VCV/Female/ada2.wav", 1, 16000, 3, 3.0),
    ("VCV/Male/apa.wav", 1, 16000, 2, 2.0),
    ("VCV/Male/123.wav", 1, 16000, 2, 1.0),  # unparsable name: skipped, as the reference does
]


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    root = tmp_path_factory.mktemp("stimuli") / "New Stimuli 9-8-2024"
    rng = np.random.default_rng(5)
    data = {}
    for rel, ch, sr, width, sec in TREE:
        n = int(sr * sec)
        x = (rng.uniform(-0.9, 0.9, (ch, n))).astype(np.float64)
        _write(root / rel, x, sr, width)
        data[rel] = (x, sr, width)
    return root, data


def test_parse_dataset_tree(tree):
    root, _ = tree
    msgs = []
    log = logging.getLogger("parse-test")
    log.addHandler(type("H", (logging.Handler,), {"emit": lambda self, r: msgs.append(r.getMessage())})())
    log.setLevel(logging.INFO)
    paths, labels, label_map, meta = parse_dataset(root, log)
    assert len(paths) == len(TREE) - 1 == len(labels) == len(meta)
    assert label_map == {lab: i for i, lab in enumerate(sorted({"da", "bi", "ga", "ada", "apa"}))}
    for p, lab, md in zip(paths, labels, meta):
        assert label_map[md["phoneme"]] == lab == label_map[extract_phoneme_label(p)]
        assert md["structure"] in ("CV", "VCV") and md["gender"] in ("male", "female")
        if md["structure"] == "CV":
            assert md["vowel_context"] in ("_a_", "_e_", "_i_", "_u_")
        else:
            assert md["vowel_context"] == "unknown"
    assert any("Skipping file: 123.wav" in m for m in msgs)
    assert any(m.startswith("Structure: CV=4, VCV=2") for m in msgs)


def test_read_wav_normalisation(tree):
    root, data = tree
    for rel, (x, sr, width) in data.items():
        got, got_sr = read_wav(root / rel)
        assert got_sr == sr and got.dtype == np.float32 and got.shape == x.shape
        q = {1: 128.0, 2: 32768.0, 3: float(1 << 23)}[width]
        assert np.abs(got - x).max() <= 0.5 / q + 1e-7, rel  # quantisation only
        assert got.min() >= -1.0 and got.max() < 1.0


def test_pad_or_trim_matches_reference_rule():
    w = np.arange(10, dtype=np.float32)[None]
    # validation: centred crop / centred pad (dataset.py:187-199)
    assert np.array_equal(pad_or_trim(w, 6, "val")[0], np.arange(2, 8))
    assert np.array_equal(pad_or_trim(w, 15, "val")[0], np.r_[np.zeros(2), np.arange(10), np.zeros(3)])
    assert pad_or_trim(w, 10, "train") is w
    import random
    rng = random.Random(3)
    for _ in range(50):
        c = pad_or_trim(w, 4, "train", rng)[0]
        assert c.shape == (4,) and np.array_equal(c, np.arange(c[0], c[0] + 4))
        p = pad_or_trim(w + 1, 13, "train", rng)[0]
        left = int(np.argmax(p != 0.0))
        assert p.shape == (13,) and np.array_equal(p[left:left + 10], np.arange(1, 11)) and p.sum() == 55


def test_from_files_val_and_train(tree):
    root, data = tree
    paths, labels, label_map, meta = parse_dataset(root)
    ms = 32000
    val = WaveformStore.from_files(paths, labels, meta, 16000, ms, "val", torch.device("cpu"))
    assert tuple(val.waves.shape) == (len(paths), ms) and not val.recrops
    for i, p in enumerate(paths):
        rel = str(p.relative_to(root))
        x, sr, _ = data[rel]
        mono = read_wav(p)[0].mean(0) if sr == 16000 else None
        row = val.waves[i].numpy()
        if mono is None:  # resampled 22.05 kHz stereo, 2.5 s -> 40000 samples, centre-cropped
            assert np.isfinite(row).all() and np.abs(row).max() > 0.1
            continue
        n = mono.shape[0]
        if n >= ms:
            s = (n - ms) // 2
            assert np.array_equal(row, mono[s:s + ms].astype(np.float32)), rel
        else:
            left = (ms - n) // 2
            assert np.array_equal(row[left:left + n], mono.astype(np.float32)), rel
            assert not row[:left].any() and not row[left + n:].any()
    tr = WaveformStore.from_files(paths, labels, meta, 16000, ms, "train", torch.device("cpu"), seed=7)
    tr2 = WaveformStore.from_files(paths, labels, meta, 16000, ms, "train", torch.device("cpu"), seed=7)
    assert torch.equal(tr.waves, tr2.waves) and not tr.recrops  # < 500 files: one cached crop
    idx = torch.arange(len(paths))
    assert torch.equal(tr.clips(idx, 0), tr.clips(idx, 3))
    for i, p in enumerate(paths):
        mono = read_wav(p)[0].mean(0).astype(np.float32)
        if read_wav(p)[1] != 16000:
            continue
        row = tr.waves[i].numpy()
        if mono.shape[0] > ms:  # a window of the clip
            starts = [s for s in range(mono.shape[0] - ms + 1) if row[0] == mono[s] and row[-1] == mono[s + ms - 1]]
            assert any(np.array_equal(row, mono[s:s + ms]) for s in starts)
        elif mono.shape[0] < ms:  # the clip at some left offset, zeros around it
            nz = np.flatnonzero(row)
            left = nz[0] - int(np.flatnonzero(mono)[0])
            assert np.array_equal(row[left:left + mono.shape[0]], mono)


def test_large_train_store_recrops_per_epoch(tmp_path):
    """>= 500 train clips: uncropped clips kept, a fresh crop / pad per epoch drawn from (seed, epoch,
    clip); same on every rank; every output a window of its clip (or the clip inside zeros)."""
    n, ms = 500, 64
    rng = np.random.default_rng(9)
    lens = rng.integers(20, 120, n)
    paths = []
    for i in range(n):
        p = tmp_path / "VCV" / "Male" / f"aba{i}.wav"
        x = rng.uniform(-0.5, 0.5, (1, lens[i]))
        x[0, 0] = x[0, -1] = 0.25  # non-zero ends locate the clip inside the pad
        _write(p, x, 16000, 2)
        paths.append(p)
    st = WaveformStore.from_files(paths, [0] * n, [{}] * n, 16000, ms, "train", torch.device("cpu"), seed=11)
    # ragged: one concatenated buffer, each clip at its own length (no [N, L_max] padding)
    assert st.recrops and st.flat.dim() == 1 and st.flat.numel() == int(lens.sum())
    assert list(st.offsets[:3]) == [0, lens[0], lens[0] + lens[1]]
    idx = torch.arange(n)
    c0, c1 = st.clips(idx, 0), st.clips(idx, 1)
    assert tuple(c0.shape) == (n, ms) and not torch.equal(c0, c1)
    assert torch.equal(c0, WaveformStore.from_files(paths, [0] * n, [{}] * n, 16000, ms, "train",
                                                    torch.device("cpu"), seed=11).clips(idx, 0))
    sub = torch.tensor([5, 17, 5])
    assert torch.equal(st.clips(sub, 1), c1[sub])  # a clip's draw does not depend on its batch
    assert torch.equal(st.clips([5, 17, 5], 1), c1[sub])  # host index lists (the loaders' form)
    part = st.subset([17, 5, 300])
    assert part.flat.numel() == int(lens[[17, 5, 300]].sum())
    assert torch.equal(part.flat[int(lens[17]):int(lens[17] + lens[5])], st.flat[st.offsets[5]:st.offsets[5] + lens[5]])
    sh = crop_shifts(lens, ms, 11, 1, np.arange(n))
    for i in range(n):
        mono = read_wav(paths[i])[0][0]
        row = c1[i].numpy()
        if lens[i] > ms:
            assert 0 <= sh[i] <= lens[i] - ms and np.array_equal(row, mono[sh[i]:sh[i] + ms])
        else:
            left = -sh[i]
            assert 0 <= left <= ms - lens[i] and np.array_equal(row[left:left + lens[i]], mono)
            assert not row[:left].any() and not row[left + lens[i]:].any()
    # the draws cover the whole range (uniform over [0, span])
    big = np.full(20000, ms + 10)
    s = crop_shifts(big, ms, 1, 0, np.arange(20000))
    assert s.min() == 0 and s.max() == 10 and abs(s.mean() - 5) < 0.1


def test_loader_epoch_follows_set_epoch(tmp_path):
    """GpuContrastiveBatches draws the crops of the epoch it is told (set_epoch, as the trainer calls
    it), not of how many passes ran: an extra pass does not shift the schedule."""
    from phoneme_contrast_amd.data import GpuContrastiveBatches
    n, ms = 8, 16
    lens = np.array([30, 5, 40, 16, 17, 9, 50, 20])
    flat = torch.arange(int(lens.sum()), dtype=torch.float32) + 1.0
    st = WaveformStore(None, [i // 2 for i in range(n)], flat=flat, lengths=lens, max_samples=ms, seed=3)

    class Ident:
        def __call__(self, clips, idx):
            return clips

    ld = GpuContrastiveBatches(st, [[0, 1, 2, 3], [4, 5, 6, 7]], Ident())
    ld.set_epoch(2)
    e2 = [b["views"].clone() for b in ld]
    list(ld)  # an extra pass (e.g. the classifier probe) ...
    ld.set_epoch(2)
    assert all(torch.equal(a, b["views"]) for a, b in zip(e2, ld))  # ... does not shift epoch 2
    ld.set_epoch(3)
    assert not all(torch.equal(a, b["views"]) for a, b in zip(e2, ld))
    assert torch.equal(e2[0], st.clips([0, 1, 2, 3], 2))
