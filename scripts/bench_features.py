#!/usr/bin/env python
"""Throughput of the on-GPU feature path: B clips of 2 s at 16 kHz ->
2 views each (random gain, MFCC 40 x 201, TimeMask + FrequencyMask + GaussianNoise), i.e. the
per-item work of PhonemeContrastiveDataset.__getitem__ (dataset.py:64-111) for a whole batch.
Prints one JSON line: views/s, per-kernel averages (HIP events), and the DFT GEMM's MFMA rate."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clips", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    from phoneme_contrast_amd import transforms as A
    from phoneme_contrast_amd.features import GpuViewBuilder, MFCCExtractor
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(0)
    wave = torch.randn(args.clips, 32000, generator=g).to(dev)
    pipe = A.build_augmentation_pipeline({"time_mask": {"enabled": True}, "freq_mask": {"enabled": True},
                                          "noise": {"enabled": True}})
    fx = MFCCExtractor().to(dev)
    vb = GpuViewBuilder(fx, pipe, n_views=2)
    idx = list(range(args.clips))
    vb(wave, idx)
    torch.cuda.synchronize()
    # device time of the kernels alone (host-side RNG draws excluded): MFCC of all views
    gain = torch.ones(2 * args.clips, device=dev)
    w2 = wave.repeat_interleave(2, 0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.steps):
        fx(w2, gain=gain, clamp_group=1)
    e1.record()
    torch.cuda.synchronize()
    dev_ms = e0.elapsed_time(e1) / args.steps
    t0 = time.perf_counter()
    for _ in range(args.steps):
        vb(wave, idx)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.steps
    nv = 2 * args.clips
    dft_flop = float(nv) * 7 * 2 * 32 * 448 * 400  # |DFT|^2 GEMM as executed (7 tiles of 32 frames, 448 cos/sin cols)
    print(json.dumps({"metric": "MFCC views/s (2 s clips, 2 views, gain + MFCC + SpecAugment)",
                      "views": nv, "wall_ms_per_batch": round(1e3 * wall, 3), "views_per_s": round(nv / wall, 1),
                      "mfcc_device_ms": round(dev_ms, 3), "mfcc_views_per_s_device": round(nv / dev_ms * 1e3, 1),
                      "dft_gemm_tflops": round(dft_flop / (dev_ms * 1e-3) / 1e12, 2)}))


if __name__ == "__main__":
    main()
