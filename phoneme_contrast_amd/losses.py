"""Contrastive losses and the loss registry — drop-in for reference src/training/losses.py.

Same class names, constructor arguments, forward signatures, reduction semantics, exceptions
and registry (`get_loss_fn`).  The arithmetic runs in libpcx (supcon.hip): one fused forward
(row max / log-sum-exp / positive sums over MFMA tiles of F F^T) and a closed-form backward.
"""
from typing import Optional

import torch
import torch.distributed as dist
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


def _all_gather_rows(local: torch.Tensor, world: int, group) -> torch.Tensor:
    """[n, ...] per rank -> [world * n, ...] in rank order (one collective)."""
    out = torch.empty((world * local.shape[0],) + tuple(local.shape[1:]), dtype=local.dtype,
                      device=local.device)
    if dist.get_backend(group) == "gloo":  # (tests / one-GPU rehearsal: gloo's list form)
        dist.all_gather(list(out.chunk(world)), local.contiguous(), group=group)
    else:
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    return out


class _GlobalSupConFn(torch.autograd.Function):
    """SupCon over the concatenation of every rank's batch (SURVEY 8(e) "global" mode).

    Forward: all-gather the [B_local, D] embeddings (and labels) into the global [B, D] batch;
    this rank's rows [r B_local, (r+1) B_local) are the anchors against all B columns
    (pcx_supcon_forward_rows); the ranks' shares of the mean/sum are all-reduced into the batch
    value (so every rank returns the same loss).  Backward: each rank turns its rowstats into
    per-anchor gradient coefficients, the [B, 4] coefficients are all-gathered (16 bytes per row)
    and pcx_supcon_backward_rows writes the FULL d loss / d F_local of this rank's rows -- the
    anchor-side and the column-side terms -- so no reduce-scatter of dF is needed.  The rank's
    parameter gradient is then its share of the global gradient: the all-reduce SUM is the
    gradient (grad_scale 1, not 1/world; ContrastiveTrainer and bench.py read `global_batch`)."""

    @staticmethod
    def forward(ctx, features, labels, mask, temperature, base_temperature, reduction, group):
        lib = _lib.lib()
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        Bl, D = features.shape
        f = features.contiguous().float()
        f_all = _all_gather_rows(f, world, group)
        lab_all = _all_gather_rows(labels.contiguous().to(torch.int64), world, group) if labels is not None else None
        msk = mask.contiguous().float() if mask is not None else None
        B, row0 = world * Bl, rank * Bl
        red = _lib.REDUCTIONS.get(reduction, 2)
        loss = torch.empty(Bl if red == 2 else 1, device=f.device, dtype=torch.float32)
        rowstats = torch.empty(Bl, 4, device=f.device, dtype=torch.float32)
        nws = lib.pcx_supcon_rows_workspace_bytes(B, D, Bl)
        ws = _lib.workspace(nws, f.device)
        _lib.check(lib.pcx_supcon_forward_rows(_lib.ptr(f_all), _lib.ptr(lab_all), _lib.ptr(msk), B, D, row0, Bl,
                                               float(temperature), float(base_temperature), red,
                                               _lib.ptr(loss), _lib.ptr(rowstats), _lib.ptr(ws), nws,
                                               _lib.stream_of(f)), "pcx_supcon_forward_rows")
        if red != 2:
            dist.all_reduce(loss, op=dist.ReduceOp.SUM, group=group)
        ctx.save_for_backward(f_all, lab_all if lab_all is not None else torch.empty(0),
                              msk if msk is not None else torch.empty(0), rowstats)
        ctx.has_lab = lab_all is not None
        ctx.cfg = (float(temperature), float(base_temperature), red, world, row0, group)
        return loss if red == 2 else loss.reshape(())

    @staticmethod
    def backward(ctx, grad_out):
        f_all, lab, msk, rowstats = ctx.saved_tensors
        lab = lab if ctx.has_lab else None
        msk = None if ctx.has_lab else msk
        t, bt, red, world, row0, group = ctx.cfg
        lib = _lib.lib()
        Bl, B, D = rowstats.shape[0], f_all.shape[0], f_all.shape[1]
        g = grad_out.contiguous().float().reshape(-1)
        coef = torch.empty(Bl, 4, device=f_all.device, dtype=torch.float32)
        stream = _lib.stream_of(f_all)
        _lib.check(lib.pcx_supcon_coef_rows(_lib.ptr(rowstats), _lib.ptr(g), B, Bl, bt, red, _lib.ptr(coef),
                                            stream), "pcx_supcon_coef_rows")
        coef_all = _all_gather_rows(coef, world, group)
        df = torch.empty(Bl, D, device=f_all.device, dtype=torch.float32)
        nws = lib.pcx_supcon_rows_workspace_bytes(B, D, Bl)
        ws = _lib.workspace(nws, f_all.device)
        _lib.check(lib.pcx_supcon_backward_rows(_lib.ptr(f_all), _lib.ptr(lab), _lib.ptr(msk), B, D, row0, Bl, t,
                                                bt, _lib.ptr(coef_all), _lib.ptr(df), _lib.ptr(ws), nws, stream),
                   "pcx_supcon_backward_rows")
        return df, None, None, None, None, None, None


class GlobalSupervisedContrastiveLoss(SupervisedContrastiveLoss):
    """SupervisedContrastiveLoss over the GLOBAL batch of a data-parallel job: every anchor sees
    the positives and negatives of all ranks, i.e. the reference loss (losses.py:41-86) on the
    concatenated batch, computed without redundancy (each rank owns its anchor rows, see
    _GlobalSupConFn).  Same constructor and forward as the reference class; `mask`, if given, is
    the global [B, B] mask (identical on every rank).  Every rank must pass the same local batch
    size.  `global_batch = True` tells the trainer to SUM (not average) the ranks' gradients.
    In a single process it is exactly SupervisedContrastiveLoss."""

    global_batch = True

    def __init__(self, temperature: float = 0.07, base_temperature: float = 0.07,
                 reduction: str = "mean", group=None):
        super().__init__(temperature, base_temperature, reduction)
        self.group = group

    def forward(self, features: torch.Tensor, labels: torch.Tensor,
                mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(self.group) == 1:
            return super().forward(features, labels, mask)
        _lib.require_gpu(features, labels, mask, what="GlobalSupervisedContrastiveLoss")
        if features.dim() != 2:
            raise ValueError(f"features must be [batch, dim], got {tuple(features.shape)}")
        world = dist.get_world_size(self.group)
        if mask is not None:
            labels = None
            if tuple(mask.shape) != (world * features.shape[0],) * 2:
                raise ValueError(f"global mode: mask must be the global [{world * features.shape[0]}]^2 mask")
        elif labels is None:
            raise ValueError("either labels or mask must be given")
        else:
            labels = labels.reshape(-1)
            if labels.shape[0] != features.shape[0]:
                raise ValueError("Num of labels does not match num of features")
        # every rank must pass the same local batch size (the gathers below need it): checked on
        # EVERY call by one 2-int collective that every rank issues, so the collectives line up
        # whatever sizes the ranks see (a per-rank "already checked" cache would let one rank skip
        # the collective while another enters it)
        n = features.shape[0]
        ext = torch.tensor([n, -n], device=features.device)  # (max, -min) in one collective
        dist.all_reduce(ext, op=dist.ReduceOp.MAX, group=self.group)
        hi, neg_lo = ext.tolist()
        if hi != -neg_lo:
            raise ValueError(f"global mode: every rank must pass the same local batch size (got {-neg_lo}..{hi})")
        return _GlobalSupConFn.apply(features, labels, mask, self.temperature, self.base_temperature,
                                     self.reduction, self.group)


class NTXentLoss(nn.Module):
    """NT-Xent; reference losses.py:89-159.  With labels it is SupCon at base_T = T; the
    label-free branch raises exactly as the reference does."""

    def __init__(self, temperature: float = 0.07, reduction: str = "mean"):
        super().__init__()
        self.temperature = temperature
        self.reduction = reduction

    def forward(self, features: torch.Tensor, labels: torch.Tensor = None) -> torch.Tensor:
        if labels is not None:
            if features.dim() == 2 and features.shape[0] == 1:
                # the reference's labelled branch has no batch-size check (losses.py:114-151): a
                # lone anchor has no positive and no other column, so its loss is -0/1 = -0.0 with
                # a zero gradient (the SupCon kernels need B >= 2)
                _lib.require_gpu(features, labels, what="NTXentLoss")
                per = -(features * 0.0).sum(dim=1)
                return per.mean() if self.reduction == "mean" else per.sum() if self.reduction == "sum" else per
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
