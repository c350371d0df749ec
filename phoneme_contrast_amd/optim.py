"""Fused Adam over one flat parameter buffer — drop-in for the reference's optimizer.

The reference builds `torch.optim.Adam(model.parameters(), lr, weight_decay)` (scripts/train.py:
129-133): coupled L2 decay, betas (0.9, 0.999), eps 1e-8, bias correction.  FusedAdam keeps that
exact update but re-homes every parameter of a group into one contiguous fp32 buffer and runs a
single libpcx kernel (pcx_adam_step) per step instead of one torch kernel chain per tensor.
`state_dict()` is laid out like torch.optim.Adam's (per-parameter step / exp_avg / exp_avg_sq),
so checkpoints written by the trainer load into either optimizer.
"""
import torch

from . import _lib


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if lr < 0.0:
            raise ValueError(f"Invalid learning rate: {lr}")
        if eps < 0.0:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError(f"Invalid beta parameters: {betas}")
        if weight_decay < 0.0:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._flat = [None] * len(self.param_groups)

    # ------------------------------------------------------------------ flat storage
    def _group_flat(self, gi):
        group = self.param_groups[gi]
        ps = group["params"]
        st = self._flat[gi]
        if st is not None and self._bound(st, ps):
            return st
        dev = ps[0].device
        _lib.require_gpu(ps[0], what="FusedAdam")
        n = sum(p.numel() for p in ps)
        flat = torch.empty(n, device=dev, dtype=torch.float32)
        m = torch.zeros(n, device=dev, dtype=torch.float32)
        v = torch.zeros(n, device=dev, dtype=torch.float32)
        step = 0
        off = 0
        # parameters re-bound behind the optimizer's back (model.to(), load_state_dict(assign=True)):
        # the moments and step count of the previous flat buffers carry over; state loaded through
        # load_state_dict (which drops the flat buffers) comes from self.state
        prev = st if st is not None and st["n"] == n else None
        for p in ps:
            k = p.numel()
            flat[off:off + k].copy_(p.detach().reshape(-1))
            s = self.state.get(p)
            if prev is not None:
                m[off:off + k].copy_(prev["m"][off:off + k])
                v[off:off + k].copy_(prev["v"][off:off + k])
                step = prev["step"]
            elif s and "exp_avg" in s:
                m[off:off + k].copy_(s["exp_avg"].reshape(-1))
                v[off:off + k].copy_(s["exp_avg_sq"].reshape(-1))
                step = int(s["step"])
            p.data = flat[off:off + k].view_as(p)
            off += k
        st = {"flat": flat, "m": m, "v": v, "step": step, "n": n, "stage": None}
        self._flat[gi] = st
        return st

    @staticmethod
    def _bound(st, ps):
        base = st["flat"].data_ptr()
        off = 0
        for p in ps:
            if p.data_ptr() != base + 4 * off:
                return False
            off += p.numel()
        return True

    @staticmethod
    def _flat_grad(st, ps):
        """The group's gradients as one flat tensor: a zero-copy view when the backward produced
        them contiguously in parameter order (libpcx does), else one gather copy."""
        g0 = ps[0].grad
        # zero-copy only when the view starts 16-byte aligned (pcx_adam_step's vector loads): a
        # second parameter group's gradients can sit at any offset of the backward's flat buffer
        if g0 is not None and g0.is_contiguous() and g0.data_ptr() % 16 == 0:
            base, sto = g0.data_ptr(), g0.untyped_storage().data_ptr()
            off, ok = 0, True
            for p in ps:
                g = p.grad
                if (g is None or not g.is_contiguous() or g.data_ptr() != base + 4 * off
                        or g.untyped_storage().data_ptr() != sto or g.dtype != torch.float32):
                    ok = False
                    break
                off += p.numel()
            if ok:
                return torch.empty(0, device=g0.device).set_(g0.untyped_storage(), g0.storage_offset(),
                                                             (st["n"],), (1,))
        if st["stage"] is None:
            st["stage"] = torch.empty_like(st["flat"])
        buf, off = st["stage"], 0
        for p in ps:
            k = p.numel()
            if p.grad is None:
                raise RuntimeError("FusedAdam: every parameter of a group needs a gradient")
            buf[off:off + k].copy_(p.grad.reshape(-1))
            off += k
        return buf

    # ------------------------------------------------------------------ step
    @torch.no_grad()
    def step(self, closure=None, flat_grads=None, grad_scale=1.0):
        """Adam step.  `flat_grads` (one flat tensor per group, e.g. after an all-reduce) bypasses
        the p.grad gather; `grad_scale` multiplies the gradient first (1/world_size)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _lib.lib()
        for gi, group in enumerate(self.param_groups):
            ps = group["params"]
            if not ps:
                continue
            st = self._group_flat(gi)
            if flat_grads is not None:
                g = flat_grads[gi]
            else:
                if all(p.grad is None for p in ps):
                    continue
                g = self._flat_grad(st, ps)
            st["step"] += 1
            b1, b2 = group["betas"]
            _lib.check(lib.pcx_adam_step(_lib.ptr(st["flat"]), _lib.ptr(g), _lib.ptr(st["m"]),
                                         _lib.ptr(st["v"]), st["n"], st["step"], float(group["lr"]),
                                         float(b1), float(b2), float(group["eps"]),
                                         float(group["weight_decay"]), float(grad_scale),
                                         _lib.stream_of(st["flat"])), "pcx_adam_step")
        return loss

    def flat_grad_views(self):
        """Flat gradient tensors (one per group), zero-copy when possible — for all-reduce."""
        out = []
        for gi, group in enumerate(self.param_groups):
            st = self._group_flat(gi)
            out.append(self._flat_grad(st, group["params"]))
        return out

    # ------------------------------------------------------------------ torch.optim.Adam-style state
    def state_dict(self):
        for gi, group in enumerate(self.param_groups):
            st = self._flat[gi]
            if st is None:
                continue
            off = 0
            for p in group["params"]:
                k = p.numel()
                self.state[p] = {"step": torch.tensor(float(st["step"])),
                                 "exp_avg": st["m"][off:off + k].view_as(p).clone(),
                                 "exp_avg_sq": st["v"][off:off + k].view_as(p).clone()}
                off += k
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._flat = [None] * len(self.param_groups)
