"""Contrastive losses and the loss registry — drop-in for reference src/training/losses.py.

Same class names, constructor arguments, forward signatures, reduction semantics, exceptions
and registry (`get_loss_fn`).  The arithmetic runs in libpcx (supcon.hip): one fused forward
(row max / log-sum-exp / positive sums over MFMA tiles of F F^T) and a closed-form backward.
"""
from typing import Optional

import torch
import torch.nn as nn

from . import _lib


class _SupConFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, features, labels, mask, temperature, base_temperature, reduction):
        lib = _lib.lib()
        B, D = features.shape
        f = features.contiguous().float()
        lab = labels.contiguous().to(torch.int64) if labels is not None else None
        msk = mask.contiguous().float() if mask is not None else None
        red = _lib.REDUCTIONS.get(reduction, 2)
        loss = torch.empty(B if red == 2 else 1, device=f.device, dtype=torch.float32)
        rowstats = torch.empty(B, 4, device=f.device, dtype=torch.float32)
        nws = lib.pcx_supcon_workspace_bytes(B, D)
        ws = _lib.workspace(nws, f.device)
        _lib.check(lib.pcx_supcon_forward(_lib.ptr(f), _lib.ptr(lab), _lib.ptr(msk), B, D,
                                          float(temperature), float(base_temperature), red,
                                          _lib.ptr(loss), _lib.ptr(rowstats), _lib.ptr(ws), nws,
                                          _lib.stream_of(f)), "pcx_supcon_forward")
        ctx.save_for_backward(f, lab if lab is not None else torch.empty(0),
                              msk if msk is not None else torch.empty(0), rowstats)
        ctx.has_lab = lab is not None
        ctx.cfg = (float(temperature), float(base_temperature), red)
        return loss if red == 2 else loss.reshape(())

    @staticmethod
    def backward(ctx, grad_out):
        f, lab, msk, rowstats = ctx.saved_tensors
        lab = lab if ctx.has_lab else None
        msk = None if ctx.has_lab else msk
        t, bt, red = ctx.cfg
        lib = _lib.lib()
        B, D = f.shape
        g = grad_out.contiguous().float().reshape(-1)
        df = torch.empty_like(f)
        nws = lib.pcx_supcon_workspace_bytes(B, D)
        ws = _lib.workspace(nws, f.device)
        _lib.check(lib.pcx_supcon_backward(_lib.ptr(f), _lib.ptr(lab), _lib.ptr(msk), B, D, t, bt,
                                           red, _lib.ptr(g), _lib.ptr(rowstats), _lib.ptr(df),
                                           _lib.ptr(ws), nws, _lib.stream_of(f)),
                   "pcx_supcon_backward")
        return df, None, None, None, None, None


def supcon(features, labels=None, mask=None, temperature=0.07, base_temperature=0.07,
           reduction="mean"):
    _lib.require_gpu(features, labels, mask, what="SupervisedContrastiveLoss")
    if features.dim() != 2:
        raise ValueError(f"features must be [batch, dim], got {tuple(features.shape)}")
    if features.shape[0] == 1:
        raise ValueError("Batch size must be greater than 1 for contrastive loss")
    if mask is not None:
        labels = None
    elif labels is None:
        raise ValueError("either labels or mask must be given")
    else:
        labels = labels.reshape(-1)
        if labels.shape[0] != features.shape[0]:
            raise ValueError("Num of labels does not match num of features")
    return _SupConFn.apply(features, labels, mask, temperature, base_temperature, reduction)


class SupervisedContrastiveLoss(nn.Module):
    """Supervised Contrastive Loss (Khosla et al., 2020); reference losses.py:8-86.

    forward(features [B,D] (L2-normalised), labels [B], mask [B,B] | None) -> scalar
    ('mean'/'sum') or per-anchor [B] (any other reduction string, as in the reference)."""

    def __init__(self, temperature: float = 0.07, base_temperature: float = 0.07,
                 reduction: str = "mean"):
        super().__init__()
        self.temperature = temperature
        self.base_temperature = base_temperature
        self.reduction = reduction

    def forward(self, features: torch.Tensor, labels: torch.Tensor,
                mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        return supcon(features, labels, mask, self.temperature, self.base_temperature,
                      self.reduction)


class NTXentLoss(nn.Module):
    """NT-Xent; reference losses.py:89-159.  With labels it is SupCon at base_T = T; the
    label-free branch raises exactly as the reference does."""

    def __init__(self, temperature: float = 0.07, reduction: str = "mean"):
        super().__init__()
        self.temperature = temperature
        self.reduction = reduction

    def forward(self, features: torch.Tensor, labels: torch.Tensor = None) -> torch.Tensor:
        if labels is not None:
            return supcon(features, labels, None, self.temperature, self.temperature,
                          self.reduction)
        if features.shape[0] % 2 != 0:
            raise ValueError("Batch size must be even for NT-Xent loss without labels")
        raise NotImplementedError("NT-Xent without labels not implemented in this version")


_LOSSES = {
    "supervised_contrastive": SupervisedContrastiveLoss,
    "ntxent": NTXentLoss,
}


def get_loss_fn(name: str, **kwargs):
    """Loss registry (reference losses.py:162-173)."""
    if name not in _LOSSES:
        raise ValueError(f"Loss {name} not found. Available: {list(_LOSSES.keys())}")
    return _LOSSES[name](**kwargs)
