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


def test_supcon_errors_match_reference():
    from phoneme_contrast_amd.losses import NTXentLoss, SupervisedContrastiveLoss
    f = torch.nn.functional.normalize(torch.randn(1, 128, device="cuda"), dim=1)
    with pytest.raises(ValueError, match="Batch size must be greater than 1"):
        SupervisedContrastiveLoss(0.5)(f, torch.tensor([0], device="cuda"))
    with pytest.raises(ValueError):
        NTXentLoss(0.5)(torch.randn(7, 128, device="cuda"))
    with pytest.raises(NotImplementedError):
        NTXentLoss(0.5)(torch.randn(8, 128, device="cuda"))


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
