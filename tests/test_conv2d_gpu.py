"""Kernel-level parity of the convolution engines behind pcx_conv2d (convg.hip / convg_bf16.hip /
convn.hip, and for fp32 stride-1 3x3 forward / data gradient with rows >= 31 columns the Winograd
F(2x2,3x3) conv of conv_wino.hip, which the networks run) against float64 torch: forward, data gradient (incl. the stride-2 parity classes) and weight
gradient at the layer shapes of PhonemeNetDeep (reference src/models/phoneme_cnn.py:146-304) and at
ragged ones.  precision 1 (bf16) is compared with the float64 result on operands rounded to bf16
first: products of bf16 values are exact in float32, so both precisions are held to the same
float32-accumulation bound, 2e-5 of the output's max |value|."""
import ctypes

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [  # B, cin, cout, IH, IW, k, stride, pad
    (2, 1, 64, 40, 33, 7, 1, 3),    # stem
    (3, 8, 16, 20, 51, 3, 2, 1),    # stride 2, channels not a multiple of 32 (general K walk)
    (2, 32, 64, 5, 26, 3, 2, 1),    # block 3 conv1 at T = 201
    (2, 64, 64, 3, 13, 3, 1, 1),
    (2, 64, 128, 10, 25, 3, 2, 1),
    (2, 16, 32, 10, 25, 1, 2, 0),   # 1x1 stride-2 shortcut
    (2, 48, 40, 7, 9, 3, 1, 1),
    # channel-last bf16 engine (convn.hip) at block shapes: 64-row and 128-row tiles, ragged tails
    (3, 64, 64, 20, 100, 3, 1, 1),
    (2, 128, 256, 10, 50, 3, 2, 1),
    (2, 256, 256, 5, 25, 3, 1, 1),
    (2, 256, 512, 5, 25, 1, 2, 0),
    # halo-staged stride-1 path (round 5, convn_halo_tiles): 4 x 2 tiles of 5 x 25 at 19 x 49 (a partial last
    # tile row and column), 11 x 11 tiles at 11 x 21 (7 idle MFMA columns), 10 x 12 tiles at 10 x 47, 128 rows
    (2, 64, 32, 19, 49, 3, 1, 1),
    (2, 32, 32, 11, 21, 3, 1, 1),
    (2, 32, 64, 10, 47, 3, 1, 1),
    (2, 128, 128, 10, 47, 3, 1, 1),
    # Winograd conv (fp32): cnn_small layer shapes, odd width (T = 201), ragged odd height / width
    (3, 32, 32, 40, 201, 3, 1, 1),
    (2, 64, 32, 20, 100, 3, 1, 1),
    (2, 32, 128, 10, 50, 3, 1, 1),
    (5, 128, 64, 9, 33, 3, 1, 1),
]


def _run(mode, prec, B, cin, cout, IH, IW, k, s, p, x, w, dy, acc=None):
    from phoneme_contrast_amd import _lib
    lib = _lib.lib()
    OH, OW = (IH + 2 * p - k) // s + 1, (IW + 2 * p - k) // s + 1
    if mode == 0:
        out = torch.empty(B, cout, OH, OW, device="cuda")
    elif mode == 1:
        out = acc.clone() if acc is not None else torch.empty(B, cin, IH, IW, device="cuda")
    else:
        out = torch.empty(cout, cin, k, k, device="cuda")
    nb = lib.pcx_conv2d_workspace_bytes(mode, prec, B, cin, cout, OH, OW, k)
    ws = torch.empty(max(nb, 4) // 4 + 1, device="cuda")
    rc = lib.pcx_conv2d(mode, prec, B, cin, cout, IH, IW, OH, OW, k, s, p, _lib.ptr(x), _lib.ptr(w), _lib.ptr(dy),
                        _lib.ptr(out), 1 if acc is not None else 0, _lib.ptr(ws), ws.numel() * 4,
                        ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    _lib.check(rc, "pcx_conv2d")
    torch.cuda.synchronize()
    return out.cpu().double()


@pytest.mark.parametrize("prec", [0, 1])
@pytest.mark.parametrize("shape", SHAPES)
def test_conv2d_modes(shape, prec):
    B, cin, cout, IH, IW, k, s, p = shape
    g = torch.Generator().manual_seed(sum(shape) + prec)
    OH, OW = (IH + 2 * p - k) // s + 1, (IW + 2 * p - k) // s + 1
    x = torch.randn(B, cin, IH, IW, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) * 0.1
    dy = torch.randn(B, cout, OH, OW, generator=g)
    prev = torch.randn(B, cin, IH, IW, generator=g)
    rd = (lambda t: t.to(torch.bfloat16).double()) if prec else (lambda t: t.double())
    xd, wd, dyd = rd(x), rd(w), rd(dy)
    ref_y = F.conv2d(xd, wd, stride=s, padding=p)
    ref_dx = torch.nn.grad.conv2d_input(x.shape, wd, dyd, stride=s, padding=p)
    ref_dw = torch.nn.grad.conv2d_weight(xd, w.shape, dyd, stride=s, padding=p)
    xc, wc, dyc = x.cuda(), w.cuda(), dy.cuda()
    got_y = _run(0, prec, B, cin, cout, IH, IW, k, s, p, xc, wc, dyc)
    got_dx = _run(1, prec, B, cin, cout, IH, IW, k, s, p, xc, wc, dyc)
    got_acc = _run(1, prec, B, cin, cout, IH, IW, k, s, p, xc, wc, dyc, acc=prev.cuda())
    got_dw = _run(2, prec, B, cin, cout, IH, IW, k, s, p, xc, wc, dyc)
    for name, got, ref in [("forward", got_y, ref_y), ("data grad", got_dx, ref_dx),
                           ("data grad +=", got_acc, ref_dx + prev.double()), ("weight grad", got_dw, ref_dw)]:
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        assert err < 2e-5, (name, shape, prec, err)
