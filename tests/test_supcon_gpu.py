"""SupCon / NT-Xent HIP kernels vs the reference's golden vectors and the float64 oracle."""
import numpy as np
import pytest
import torch

from golden_util import load
from oracle import np_ops as op

pytestmark = pytest.mark.gpu

CASES = sorted({k.split("/")[0] for k in load("supcon").files})


def _loss_mod(kind, T, bT, red):
    from phoneme_contrast_amd.losses import NTXentLoss, SupervisedContrastiveLoss
    if kind == "supcon":
        return SupervisedContrastiveLoss(temperature=T, base_temperature=bT, reduction=red)
    return NTXentLoss(temperature=T, reduction=red)


@pytest.mark.parametrize("case", CASES)
def test_supcon_matches_golden(case):
    d = load("supcon")
    B, D, T, bT = d[case + "/meta"]
    kind, red = str(d[case + "/kind"]), str(d[case + "/reduction"])
    f = torch.tensor(d[case + "/features"], device="cuda", requires_grad=True)
    lab = torch.tensor(d[case + "/labels"], device="cuda")
    fn = _loss_mod(kind, float(T), float(bT), red)
    if case + "/mask" in d.files:
        loss = fn(f, lab, mask=torch.tensor(d[case + "/mask"], device="cuda"))
    else:
        loss = fn(f, lab)
    (loss.sum() if loss.dim() else loss).backward()
    got_l = np.atleast_1d(loss.detach().cpu().numpy())
    ref_l = d[case + "/loss"]
    assert np.abs(got_l - ref_l).max() <= 1e-4 * max(1.0, np.abs(ref_l).max() / 10)
    ref_g = d[case + "/grad"]
    got_g = f.grad.cpu().numpy()
    assert np.abs(got_g - ref_g).max() <= 1e-4 * np.abs(ref_g).max() + 1e-7


@pytest.mark.parametrize("B,D,T", [(4096, 128, 0.15), (1000, 64, 0.07), (333, 256, 0.5)])
def test_supcon_large_vs_oracle(B, D, T):
    g = torch.Generator().manual_seed(B)
    f = torch.nn.functional.normalize(torch.randn(B, D, generator=g), dim=1)
    lab = torch.arange(B // 4 + 1).repeat_interleave(4)[:B]
    ref_l, ref_g = op.supcon_fwd_bwd(f.double().numpy(), lab.numpy(), None, T, 0.07, "mean")
    fd = f.cuda().requires_grad_(True)
    from phoneme_contrast_amd.losses import SupervisedContrastiveLoss
    loss = SupervisedContrastiveLoss(temperature=T)(fd, lab.cuda())
    loss.backward()
    assert abs(loss.item() - ref_l) < 1e-4
    err = np.abs(fd.grad.cpu().double().numpy() - ref_g).max() / np.abs(ref_g).max()
    assert err < 1e-4


@pytest.mark.parametrize("B,D,cuts,red,use_mask", [(1000, 128, (0, 333, 1000), "mean", False),
                                                   (4096, 128, (0, 512, 4096), "sum", False),
                                                   (200, 64, (0, 7, 120, 200), "none", True),
                                                   (130, 256, (0, 65, 130), "mean", True)])
def test_supcon_row_ranges_match_oracle(B, D, cuts, red, use_mask):
    """The global-batch mode's C-ABI (pcx_supcon_forward_rows / _coef_rows / _backward_rows) on a
    partition of the anchors, in one process: each range's rowstats and loss share, its gradient
    coefficients and -- given all ranges' coefficients -- the full gradient of its rows, vs the
    float64 restatement (oracle/np_ops.py supcon_rows_*), and the assembled ranges vs the
    single-batch reference loss."""
    from phoneme_contrast_amd import _lib
    lib = _lib.lib()
    g = torch.Generator().manual_seed(B + D)
    f = torch.nn.functional.normalize(torch.randn(B, D, generator=g), dim=1)
    lab = torch.randint(0, max(2, B // 5), (B,), generator=g)
    mask = (torch.rand(B, B, generator=g) < 0.05).float() if use_mask else None
    T, bT = 0.12, 0.07
    red_i = _lib.REDUCTIONS[red]
    fd = f.cuda()
    labd = None if use_mask else lab.cuda()
    maskd = mask.cuda() if use_mask else None
    stream = _lib.stream_of(fd)
    ranges = list(zip(cuts[:-1], cuts[1:]))
    shares, coefs, stats = [], [], []
    for lo, hi in ranges:
        n = hi - lo
        loss = torch.empty(n if red == "none" else 1, device="cuda")
        st = torch.empty(n, 4, device="cuda")
        nws = lib.pcx_supcon_rows_workspace_bytes(B, D, n)
        ws = _lib.workspace(nws, fd.device)
        _lib.check(lib.pcx_supcon_forward_rows(_lib.ptr(fd), _lib.ptr(labd), _lib.ptr(maskd), B, D, lo, n, T, bT,
                                               red_i, _lib.ptr(loss), _lib.ptr(st), _lib.ptr(ws), nws, stream), "fwd")
        gout = torch.ones(n if red == "none" else 1, device="cuda")
        cf = torch.empty(n, 4, device="cuda")
        _lib.check(lib.pcx_supcon_coef_rows(_lib.ptr(st), _lib.ptr(gout), B, n, bT, red_i, _lib.ptr(cf), stream),
                   "coef")
        shares.append(loss.cpu().double().numpy())
        stats.append(st.cpu().double().numpy())
        coefs.append(cf)
    coef_all = torch.cat(coefs)
    fn, mn, ln = f.double().numpy(), (mask.double().numpy() if use_mask else None), lab.numpy()
    ref_l, ref_g = op.supcon_fwd_bwd(fn, None if use_mask else ln, mn, T, bT, red)
    cref = []
    for (lo, hi), share, st in zip(ranges, shares, stats):
        s_ref, st_ref = op.supcon_rows_fwd(fn, None if use_mask else ln, mn, lo, hi - lo, T, bT, red)
        assert np.abs(share - s_ref).max() <= 1e-4 * max(1.0, np.abs(s_ref).max())
        assert np.abs(st[:, 3] - st_ref[:, 3]).max() <= 1e-4 * max(1.0, np.abs(st_ref[:, 3]).max())
        cref.append(op.supcon_coef_rows(st_ref, np.ones(hi - lo if red == "none" else 1), B, bT, red))
    got_l = np.concatenate(shares) if red == "none" else sum(s[0] for s in shares)
    assert np.abs(got_l - ref_l).max() <= 1e-4 * max(1.0, np.abs(ref_l).max())
    np.testing.assert_allclose(coef_all.cpu().double().numpy()[:, :3], np.concatenate(cref), rtol=1e-4, atol=1e-9)
    parts = []
    for lo, hi in ranges:
        n = hi - lo
        df = torch.empty(n, D, device="cuda")
        nws = lib.pcx_supcon_rows_workspace_bytes(B, D, n)
        ws = _lib.workspace(nws, fd.device)
        _lib.check(lib.pcx_supcon_backward_rows(_lib.ptr(fd), _lib.ptr(labd), _lib.ptr(maskd), B, D, lo, n, T, bT,
                                                _lib.ptr(coef_all), _lib.ptr(df), _lib.ptr(ws), nws, stream), "bwd")
        parts.append(df.cpu().double().numpy())
    got_g = np.concatenate(parts)
    assert np.abs(got_g - ref_g).max() <= 1e-4 * np.abs(ref_g).max() + 1e-7


def test_supcon_row_range_errors():
    from phoneme_contrast_amd import _lib
    lib = _lib.lib()
    f = torch.zeros(16, 128, device="cuda")
    lab = torch.zeros(16, dtype=torch.int64, device="cuda")
    out = torch.empty(4, device="cuda")
    rc = lib.pcx_supcon_forward_rows(_lib.ptr(f), _lib.ptr(lab), None, 16, 128, 10, 8, 0.1, 0.07, 0,
                                     _lib.ptr(out), _lib.ptr(out), None, 0, _lib.stream_of(f))
    assert rc != 0 and "outside the batch" in _lib.last_error()


def test_supcon_errors_match_reference():
    from phoneme_contrast_amd.losses import NTXentLoss, SupervisedContrastiveLoss
    f = torch.nn.functional.normalize(torch.randn(1, 128, device="cuda"), dim=1)
    with pytest.raises(ValueError, match="Batch size must be greater than 1"):
        SupervisedContrastiveLoss(0.5)(f, torch.tensor([0], device="cuda"))
    with pytest.raises(ValueError):
        NTXentLoss(0.5)(torch.randn(7, 128, device="cuda"))
    with pytest.raises(NotImplementedError):
        NTXentLoss(0.5)(torch.randn(8, 128, device="cuda"))


def test_ntxent_labelled_single_sample_is_zero_like_reference():
    """The reference's labelled NT-Xent has no batch-size check (losses.py:114-151): at B = 1 the
    anchor has no positive, so every reduction gives 0 (-0.0) and the gradient is zero."""
    from phoneme_contrast_amd.losses import NTXentLoss
    for red, shape in (("mean", ()), ("sum", ()), ("none", (1,))):
        f = torch.nn.functional.normalize(torch.randn(1, 128, device="cuda"), dim=1).requires_grad_(True)
        loss = NTXentLoss(0.5, reduction=red)(f, torch.tensor([3], device="cuda"))
        assert tuple(loss.shape) == shape and float(loss.sum()) == 0.0
        loss.sum().backward()
        assert f.grad is not None and not f.grad.any()
    # and B = 2 still runs the kernel (matches SupCon at base_T = T)
    f = torch.nn.functional.normalize(torch.randn(2, 64, device="cuda"), dim=1)
    lab = torch.tensor([1, 1], device="cuda")
    s = float(NTXentLoss(0.5)(f, lab))
    ref = -(float((f[0] * f[1]).sum()) / 0.5 - np.log(np.exp(float((f[0] * f[1]).sum()) / 0.5
                                                                - 1.0 / 0.5) + 1e-6) - 1.0 / 0.5)
    assert abs(s - ref) < 1e-4


def test_adam_kernel_matches_torch():
    from phoneme_contrast_amd import _lib
    n = 304225
    g = torch.Generator().manual_seed(0)
    p0 = torch.randn(n, generator=g)
    p = p0.clone().cuda()
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    ref = p0.clone().double().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=3e-4, weight_decay=1e-4)
    for step in range(1, 4):
        gr = torch.randn(n, generator=g) * 10 ** torch.empty(n).uniform_(-6, 0, generator=g)
        ref.grad = gr.double()
        opt.step()
        gd = gr.cuda()
        _lib.check(_lib.lib().pcx_adam_step(_lib.ptr(p), _lib.ptr(gd), _lib.ptr(m), _lib.ptr(v), n,
                                            step, 3e-4, 0.9, 0.999, 1e-8, 1e-4, 1.0,
                                            _lib.stream_of(p)), "adam")
    err = (p.cpu().double() - ref.detach()).abs().max().item()
    assert err < 1e-6
