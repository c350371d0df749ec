"""Micro-benchmark of one cnn_deep convolution through pcx_conv2d (precision 0 fp32 / 1 bf16):
average time per call over --iters calls (all kernels of the call: conversion, packing, GEMM).
Usage: python tools/convn_bench.py --mode 0 --prec 1 --shape B,cin,cout,IH,IW,k,stride,pad"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from phoneme_contrast_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", type=int, default=0)
    ap.add_argument("--prec", type=int, default=1)
    ap.add_argument("--shape", default="4096,64,64,20,100,3,1,1")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--lib", default=None, help="alternative build of libpcx.so (experiments)")
    a = ap.parse_args()
    if a.lib:
        _lib.LIB_PATH = os.path.abspath(a.lib)
    B, cin, cout, IH, IW, k, s, p = map(int, a.shape.split(","))
    OH, OW = (IH + 2 * p - k) // s + 1, (IW + 2 * p - k) // s + 1
    lib = _lib.lib()
    x = torch.randn(B, cin, IH, IW, device="cuda")
    w = torch.randn(cout, cin, k, k, device="cuda") * 0.1
    dy = torch.randn(B, cout, OH, OW, device="cuda")
    out = {0: torch.empty(B, cout, OH, OW, device="cuda"), 1: torch.empty(B, cin, IH, IW, device="cuda"),
           2: torch.empty(cout, cin, k, k, device="cuda")}[a.mode]
    nb = lib.pcx_conv2d_workspace_bytes(a.mode, a.prec, B, cin, cout, OH, OW, k)
    ws = torch.empty(max(nb, 4) // 4 + 1, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    def call():
        rc = lib.pcx_conv2d(a.mode, a.prec, B, cin, cout, IH, IW, OH, OW, k, s, p, _lib.ptr(x), _lib.ptr(w),
                            _lib.ptr(dy), _lib.ptr(out), 0, _lib.ptr(ws), ws.numel() * 4, stream)
        _lib.check(rc, "pcx_conv2d")

    call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        call()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    flops = 2.0 * B * OH * OW * cout * cin * k * k
    print("mode %d prec %d shape %s: %.3f ms/call  %.1f TFLOP/s (whole call)" % (a.mode, a.prec, a.shape, ms,
                                                                                flops / ms / 1e9))


if __name__ == "__main__":
    main()
