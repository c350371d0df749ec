"""PhonemeNetDeep (cnn_deep) train step on the GPU (libpcx) vs the reference's golden vectors.

Reference: src/models/phoneme_cnn.py:146-304.  Fixtures use the full topology at reduced widths
(hidden_dims [8, 16, 32, 64]); tolerances as tests/test_model_gpu.py.  The use_residual=false
branch (phoneme_cnn.py:230-243) has no reference fixture: it is checked against a float64 PyTorch
evaluation of the same modules with the same Dropout2d masks."""
import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from golden_util import bn_fed_bias, grad_errors, model_case

pytestmark = pytest.mark.gpu

DEEP = {"in_channels": 1, "embedding_dim": 128, "use_attention": True, "dropout_rate": 0.2,
        "hidden_dims": [8, 16, 32, 64], "use_residual": True}


def _model(name, cfg=DEEP):
    from phoneme_contrast_amd.models import model_registry
    c = model_case(name)
    m = model_registry.create("phoneme_cnn_deep", cfg)
    m.load_state_dict({k: torch.tensor(v) for k, v in c["state0"].items()})
    return m.cuda().train(), c


def _step(m, c, step=0, labels=None):
    from phoneme_contrast_amd.losses import SupervisedContrastiveLoss
    m.set_dropout_masks([torch.tensor(k) for k in c["steps"][step]["masks"]])
    e = m(torch.tensor(c["x"]).cuda())
    lab = torch.tensor(c["labels"] if labels is None else labels).cuda()
    loss = SupervisedContrastiveLoss(temperature=c["temperature"])(e, lab)
    for p in m.parameters():
        p.grad = None
    loss.backward()
    return e, loss


def _check_grads(m, c):
    got = {k: p.grad.detach().cpu().numpy() for k, p in m.named_parameters()}
    e32 = grad_errors(got, c["grads"])
    e64 = grad_errors(got, c["f64"]["grads"])
    bad = {k: (e32[k], e64[k]) for k in e32
           if min(e32[k][1], e64[k][1]) > (2e-3 if e32[k][0] == "rel" else 1e-4)}
    assert not bad, bad


@pytest.mark.parametrize("name", ["cnn_deep_T200", "cnn_deep_T201"])
def test_deep_train_step_matches_reference(name):
    m, c = _model(name)
    assert len(c["steps"][0]["masks"]) == 4
    e, loss = _step(m, c)
    e = e.detach().cpu().numpy()
    assert np.abs(e - c["f64"]["emb"]).max() < 1e-5
    assert abs(loss.item() - c["f64"]["loss"]) < 1e-4
    _check_grads(m, c)


def test_deep_two_steps_with_fused_adam_track_reference():
    from phoneme_contrast_amd.optim import FusedAdam
    m, c = _model("cnn_deep_T200")
    opt = FusedAdam(m.parameters(), lr=c["lr"], weight_decay=c["weight_decay"])
    _step(m, c, 0)
    opt.step()
    _, loss = _step(m, c, 1)
    assert abs(loss.item() - c["steps"][1]["loss"]) < 2e-3
    opt.step()
    lr = c["lr"]
    for k, v in m.state_dict().items():
        ref = c["state_final"][k]
        if k.endswith("num_batches_tracked"):
            assert int(v) == int(ref), k
            continue
        diff = np.abs(v.cpu().numpy().astype(np.float64) - ref)
        tol = 1e-3 * max(1.0, np.abs(ref).max()) if "running" in k else 4 * lr + 1e-5
        assert diff.max() <= tol, (k, diff.max())


def _torch_reference(m, x, masks, margins=None):
    """float64 evaluation of PhonemeNetDeep built from the model's own nn modules (a reference
    layer-for-layer restatement of phoneme_cnn.py:274-304 with explicit Dropout2d masks).
    `margins` (a list) collects min |pre-activation| of every ReLU: how far the case sits from a
    kink where float32 rounding may legitimately flip a ReLU mask."""
    def relu(v):
        if margins is not None:
            margins.append(v.detach().abs().min().item())
        return F.relu(v)

    def seq(mod, v):
        for layer in mod:
            v = relu(v) if isinstance(layer, nn.ReLU) else layer(v)
        return v

    x = seq(m.init_conv, x) if isinstance(m.init_conv, nn.Sequential) else m.init_conv(x)
    for blk, mk in zip(m.conv_blocks, masks):
        if isinstance(blk, nn.Sequential):  # use_residual = false
            for layer in blk:
                if isinstance(layer, nn.Dropout2d):
                    x = x * mk[:, :, None, None]
                else:
                    x = relu(x) if isinstance(layer, nn.ReLU) else layer(x)
        else:
            out = relu(blk.bn1(blk.conv1(x))) * mk[:, :, None, None]
            out = blk.bn2(blk.conv2(out))
            sc = blk.shortcut(x) if len(blk.shortcut) else x
            x = relu(out + sc)
    if m.use_attention:
        x = x * torch.sigmoid(m.attention.conv(x))
    x = m.projection(x.mean(dim=(2, 3)))
    return F.normalize(x, p=2, dim=1)


FULL = [64, 128, 256, 512]  # the benchmarked widths: stride-1 3x3 convs on the LDS-DMA / 32x32 engines


# (False, 201) uses seed 5: with seed 3 one block-3 pre-activation sits 2.8e-7 from the ReLU kink
# (float64 reference, 312 values per channel there), so float32 summation order alone decides that
# mask bit and with it ~5 % of block 3's BN1 beta gradient -- measured: the forward matches to 6e-7
# and only beta (not gamma: xhat = 0 at the kink with beta = 0) moves.  Not a property of the kernels.
@pytest.mark.parametrize("residual,T,dims,B,seed", [(False, 200, None, 8, 3), (False, 201, None, 8, 5),
                                                    (True, 57, None, 8, 3), (True, 200, FULL, 4, 3),
                                                    (True, 57, FULL, 5, 3)])
def test_deep_matches_float64_torch(residual, T, dims, B, seed):
    from phoneme_contrast_amd.losses import SupervisedContrastiveLoss
    torch.manual_seed(seed)
    cfg = dict(DEEP, use_residual=residual)
    if dims:
        cfg["hidden_dims"] = dims
    from phoneme_contrast_amd.models import PhonemeNetDeep
    m = PhonemeNetDeep(cfg)
    ref = PhonemeNetDeep(cfg).double()
    ref.load_state_dict(m.state_dict())
    m = m.cuda().train()
    x = torch.randn(B, 1, 40, T)
    labels = torch.arange(B) % 4
    masks = [(torch.rand(B, c) > 0.2).float() / 0.8 for c in cfg["hidden_dims"]]
    m.set_dropout_masks(masks)
    e = m(x.cuda())
    loss = SupervisedContrastiveLoss(temperature=0.15)(e, labels.cuda())
    loss.backward()
    ref.train()
    xr = x.double().requires_grad_(False)
    margins = []
    er = _torch_reference(ref, xr, [k.double() for k in masks], margins)
    from oracle import torch_port as tp
    lr_ = tp.supcon(er, labels, 0.15, 0.07)
    lr_.backward()
    emb_err = (e.detach().cpu().double() - er.detach()).abs().max().item()
    print(f"deep residual={residual} T={T} dims={dims} B={B}: max |d emb| {emb_err:.2e}, "
          f"|d loss| {abs(loss.item() - lr_.item()):.2e}, min ReLU margin {min(margins):.1e}")
    # full widths (512 channels through 4 train-mode BN layers over B = 4 samples) condition the
    # fp32 forward worse: the general implicit-GEMM engine alone measures 1.26e-5 on (200, FULL, 4),
    # the routed engines 1.41e-5 -- float32 rounding, not a layout error, so the bound is 5e-5 there
    assert emb_err < (5e-5 if dims == FULL else 1e-5)
    assert abs(loss.item() - lr_.item()) < 1e-4
    for (k, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        g, r = p.grad.cpu().double(), q.grad
        if bn_fed_bias(k, None):
            assert g.abs().max() < 1e-4, k
            continue
        err = (g - r).abs().max() / max(r.abs().max().item(), 1e-30)
        assert err < 2e-3, (k, float(err))
    # running statistics follow torch's update
    for (k, v), (_, w) in zip(m.state_dict().items(), ref.state_dict().items()):
        if "running" in k:
            assert torch.allclose(v.cpu().double(), w, rtol=1e-5, atol=1e-6), k


def test_deep_eval_and_shapes():
    from phoneme_contrast_amd.models import PhonemeNetDeep
    torch.manual_seed(0)
    m = PhonemeNetDeep({"embedding_dim": 64, "hidden_dims": [8, 16, 32, 64]})
    ref = PhonemeNetDeep({"embedding_dim": 64, "hidden_dims": [8, 16, 32, 64]}).double()
    ref.load_state_dict(m.state_dict())
    m = m.cuda().eval()
    ref.eval()
    for bs in (1, 3):
        x = torch.randn(bs, 1, 40, 100)
        with torch.no_grad():
            e = m(x.cuda()).cpu()
            r = _torch_reference(ref, x.double(), [torch.ones(bs, c).double() for c in (8, 16, 32, 64)])
        assert e.shape == (bs, 64)
        assert (e.double() - r).abs().max() < 1e-5
        assert torch.allclose(e.norm(dim=1), torch.ones(bs), atol=1e-6)


def test_deep_fp32_full_size_properties():
    """config 3 (cnn_deep fp32, B = 4096, T = 200, widths 64..512) at its full size, where the float64
    oracle is out of reach: unit-norm finite embeddings, finite gradients, a bit-identical repeat (no
    atomics on the path), and in eval mode (running BN statistics: samples independent) the first
    8 embeddings of the 4096-batch equal those of an 8-sample batch -- a tiling / sample-boundary
    check of every conv engine at the full shapes (the float64 parity itself is the small-batch
    tests above)."""
    from phoneme_contrast_amd.losses import SupervisedContrastiveLoss
    from phoneme_contrast_amd.models import PhonemeNetDeep
    torch.manual_seed(0)
    m = PhonemeNetDeep({"embedding_dim": 128}).cuda().train()
    B = 4096
    x = torch.randn(B, 1, 40, 200, generator=torch.Generator().manual_seed(1)).cuda()
    labels = (torch.arange(B) // 4).cuda()
    masks = [(torch.rand(B, c) > 0.2).float() / 0.8 for c in m.hidden_dims]
    fn = SupervisedContrastiveLoss(temperature=0.15)
    outs = []
    for _ in range(2):
        m.zero_grad(set_to_none=True)
        m.set_dropout_masks(masks)
        e = m(x)
        loss = fn(e, labels)
        loss.backward()
        outs.append((e.detach().clone(), loss.item(), [p.grad.clone() for p in m.parameters()]))
    e, l, g = outs[0]
    assert torch.allclose(e.norm(dim=1), torch.ones(B, device=e.device), atol=1e-5)
    assert torch.isfinite(torch.tensor(l)) and all(torch.isfinite(t).all() for t in g)
    assert any(t.abs().max() > 0 for t in g)
    e2, l2, g2 = outs[1]
    assert torch.equal(e, e2) and l == l2 and all(torch.equal(a, b) for a, b in zip(g, g2))
    m.eval()
    with torch.no_grad():
        full = m(x)[:8]
        part = m(x[:8].contiguous())
    assert torch.isfinite(full).all()
    assert (full - part).abs().max().item() < 1e-5
