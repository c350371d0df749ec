"""Global-batch SupCon (SURVEY 8(e) optional mode), host side: the row-range decomposition that
pcx_supcon_forward_rows / _coef_rows / _backward_rows implement, restated in float64
(oracle/np_ops.py supcon_rows_*), reproduces the reference loss on the whole batch
(src/training/losses.py:41-86) and its gradient for every partition of the anchors -- the claim
that makes one embedding all-gather + one coefficient all-gather enough (no dF reduce-scatter).
The kernels themselves are checked against these functions in tests/test_supcon_gpu.py and, over
two ranks, in tests/test_ddp_gpu.py."""
import numpy as np
import pytest

from oracle import np_ops as op


def _batch(B, D, seed, ncls):
    rng = np.random.default_rng(seed)
    f = rng.standard_normal((B, D))
    f /= np.linalg.norm(f, axis=1, keepdims=True)
    return f, rng.integers(0, ncls, B)


@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
@pytest.mark.parametrize("cuts", [(0, 24), (0, 12, 24), (0, 5, 6, 17, 24)])
def test_row_ranges_reproduce_single_batch(reduction, cuts):
    f, lab = _batch(24, 16, len(cuts), 5)
    T, bT = 0.1, 0.07
    ref_l, ref_g = op.supcon_fwd_bwd(f, lab, None, T, bT, reduction)
    shares, coefs = [], []
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        share, st = op.supcon_rows_fwd(f, lab, None, lo, hi - lo, T, bT, reduction)
        shares.append(np.atleast_1d(share))
        g = np.ones(hi - lo) if reduction == "none" else np.ones(1)
        coefs.append(op.supcon_coef_rows(st, g, 24, bT, reduction))
    got_l = np.concatenate(shares) if reduction == "none" else sum(s[0] for s in shares)
    np.testing.assert_allclose(got_l, ref_l, rtol=1e-12, atol=1e-12)
    coef_all = np.concatenate(coefs)
    got_g = np.concatenate([op.supcon_rows_bwd(f, lab, None, lo, hi - lo, coef_all, T)
                            for lo, hi in zip(cuts[:-1], cuts[1:])])
    np.testing.assert_allclose(got_g, ref_g, rtol=1e-10, atol=1e-12)


def test_row_ranges_with_mask_and_lonely_anchor():
    """An explicit (asymmetric) mask and an anchor without positives (divides by 1, still counted)."""
    f, _ = _batch(10, 8, 3, 2)
    rng = np.random.default_rng(9)
    mask = (rng.random((10, 10)) < 0.3).astype(np.float64)
    mask[4] = 0.0
    ref_l, ref_g = op.supcon_fwd_bwd(f, None, mask, 0.2, 0.07, "mean")
    parts = [(0, 4), (4, 3), (7, 3)]
    sts = [op.supcon_rows_fwd(f, None, mask, lo, n, 0.2, 0.07, "mean") for lo, n in parts]
    assert abs(sum(s for s, _ in sts) - ref_l) < 1e-12
    coef_all = np.concatenate([op.supcon_coef_rows(st, np.ones(1), 10, 0.07, "mean") for _, st in sts])
    got = np.concatenate([op.supcon_rows_bwd(f, None, mask, lo, n, coef_all, 0.2) for lo, n in parts])
    np.testing.assert_allclose(got, ref_g, rtol=1e-10, atol=1e-12)


def test_global_loss_differs_from_per_rank_average():
    """The mode is a real semantic choice: per-rank SupCon (DDP-equivalent, the default) sees only
    local negatives, so its averaged loss differs from the global-batch loss."""
    f, lab = _batch(32, 16, 1, 4)
    glob, _ = op.supcon_fwd_bwd(f, lab, None, 0.1, 0.07, "mean")
    per = np.mean([op.supcon_fwd_bwd(f[r * 16:(r + 1) * 16], lab[r * 16:(r + 1) * 16], None, 0.1, 0.07)[0]
                   for r in range(2)])
    assert abs(glob - per) > 1e-3
