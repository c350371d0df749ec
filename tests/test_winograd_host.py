"""Host-side check of the Winograd F(2x2,3x3) algebra used by csrc/conv_wino.hip (no GPU): the
weight transform of wino_pack_kernel (incl. the data-gradient flip), the input transform of the
K-step (rows first, then columns) and the output transform of the epilogue, restated in float64
numpy with the kernel's exact operation order and tiling (2x2 output tiles, 4x4 patches starting
at (2 tr - 1, 2 tc - 1), outputs past an odd edge dropped), against the direct 3x3 / pad 1
correlation of the reference's nn.Conv2d layers (src/models/phoneme_cnn.py:29-47) and its data
gradient.  The GPU kernel itself is checked against float64 torch in tests/test_conv2d_gpu.py and
through the model golden tests."""
import numpy as np
import pytest


def weight_transform(g):
    """U = G g G^T as wino_pack_kernel evaluates it (g: [..., 3, 3])."""
    t = np.stack([g[..., 0, :], 0.5 * (g[..., 0, :] + g[..., 1, :] + g[..., 2, :]),
                  0.5 * (g[..., 0, :] - g[..., 1, :] + g[..., 2, :]), g[..., 2, :]], axis=-2)
    return np.stack([t[..., 0], 0.5 * (t[..., 0] + t[..., 1] + t[..., 2]),
                     0.5 * (t[..., 0] - t[..., 1] + t[..., 2]), t[..., 2]], axis=-1)


def input_transform(d):
    """V = B^T d B for d [..., 4, 4] in the K-step's order (row combinations, then columns)."""
    e = np.stack([d[..., 0, :] - d[..., 2, :], d[..., 1, :] + d[..., 2, :],
                  d[..., 2, :] - d[..., 1, :], d[..., 1, :] - d[..., 3, :]], axis=-2)
    return np.stack([e[..., 0] - e[..., 2], e[..., 1] + e[..., 2],
                     e[..., 2] - e[..., 1], e[..., 1] - e[..., 3]], axis=-1)


def output_transform(m):
    """Y = A^T m A for m [..., 4, 4] as the epilogue evaluates it -> [..., 2, 2]."""
    s0 = m[..., 0, :] + m[..., 1, :] + m[..., 2, :]
    s1 = m[..., 1, :] - m[..., 2, :] - m[..., 3, :]
    y0 = np.stack([s0[..., 0] + s0[..., 1] + s0[..., 2], s0[..., 1] - s0[..., 2] - s0[..., 3]], axis=-1)
    y1 = np.stack([s1[..., 0] + s1[..., 1] + s1[..., 2], s1[..., 1] - s1[..., 2] - s1[..., 3]], axis=-1)
    return np.stack([y0, y1], axis=-2)


def wino_conv(x, w):
    """x [C, H, W], w [M, C, 3, 3] -> [M, H, W] through per-element GEMMs over C."""
    C, H, W = x.shape
    TR, TC = (H + 1) // 2, (W + 1) // 2
    xp = np.zeros((C, 2 * TR + 2, 2 * TC + 2))
    xp[:, 1:H + 1, 1:W + 1] = x
    U = weight_transform(w)                                   # [M, C, 4, 4]
    out = np.zeros((w.shape[0], 2 * TR, 2 * TC))
    for tr in range(TR):
        for tc in range(TC):
            V = input_transform(xp[:, 2 * tr:2 * tr + 4, 2 * tc:2 * tc + 4])    # [C, 4, 4]
            M = np.einsum("mcij,cij->mij", U, V)               # 16 GEMMs over the channels
            out[:, 2 * tr:2 * tr + 2, 2 * tc:2 * tc + 2] = output_transform(M)
    return out[:, :H, :W]


def direct_conv(x, w):
    C, H, W = x.shape
    xp = np.pad(x, ((0, 0), (1, 1), (1, 1)))
    out = np.zeros((w.shape[0], H, W))
    for dh in range(3):
        for dw in range(3):
            out += np.einsum("mc,chw->mhw", w[:, :, dh, dw], xp[:, dh:dh + H, dw:dw + W])
    return out


@pytest.mark.parametrize("C,M,H,W", [(3, 5, 8, 10), (2, 4, 7, 9), (4, 2, 5, 33), (1, 3, 2, 2)])
def test_winograd_forward_matches_direct(C, M, H, W):
    rng = np.random.default_rng(C * 100 + H * 10 + W)
    x = rng.standard_normal((C, H, W))
    w = rng.standard_normal((M, C, 3, 3))
    np.testing.assert_allclose(wino_conv(x, w), direct_conv(x, w), rtol=0, atol=1e-12)


@pytest.mark.parametrize("C,M,H,W", [(3, 5, 8, 10), (2, 6, 9, 7)])
def test_winograd_data_gradient_flip(C, M, H, W):
    """The data gradient runs the same kernel on dy with weights flipped as wino_pack_kernel(flip=1)
    reads them: g[m][k] = w[k][m] rotated 180 degrees (m = input channel of the forward)."""
    rng = np.random.default_rng(7 + H + W)
    dy = rng.standard_normal((M, H, W))
    w = rng.standard_normal((M, C, 3, 3))                     # forward weights [cout][cin]
    g = np.transpose(w, (1, 0, 2, 3))[:, :, ::-1, ::-1]        # [cin][cout], rotated
    # reference: dx = conv_transpose of dy with w (the adjoint of the forward correlation)
    dx = np.zeros((C, H + 2, W + 2))
    for dh in range(3):
        for dw in range(3):
            dx[:, dh:dh + H, dw:dw + W] += np.einsum("mc,mhw->chw", w[:, :, dh, dw], dy)
    np.testing.assert_allclose(wino_conv(dy, np.ascontiguousarray(g)), dx[:, 1:H + 1, 1:W + 1], rtol=0, atol=1e-12)


def test_winograd_float32_error_is_small():
    """In float32 the transforms add a few ulps over the direct correlation (kernel-level GPU
    measurements: 2-6e-6 of max|y| at K = 32..1152)."""
    rng = np.random.default_rng(3)
    x = rng.standard_normal((32, 12, 20)).astype(np.float32)
    w = (0.1 * rng.standard_normal((8, 32, 3, 3))).astype(np.float32)
    ref = direct_conv(x.astype(np.float64), w.astype(np.float64))
    got = wino_conv(x, w.astype(np.float32).astype(np.float64).astype(np.float32))
    assert np.abs(got - ref).max() / np.abs(ref).max() < 1e-5
