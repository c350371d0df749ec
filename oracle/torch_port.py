"""float32 torch-CPU restatement of the phoneme-contrast train step (test oracle / CPU baseline).

Functional (no nn.Module tree): parameters live in a reference-format state_dict, the graph is
written with torch.nn.functional ops and differentiated by autograd.  Used
  * as the timed CPU baseline of bench.py ("kind": "port"), since the reference itself cannot
    travel to the GPU box, and
  * by the GPU tests to expose intermediate activations / gradients for localisation.
It is pinned against the reference's golden fixtures in tests/test_oracle_golden.py.

Reference: src/models/phoneme_cnn.py:10-304, src/training/losses.py:41-86,
scripts/train.py:128-133 (Adam), src/training/trainer.py:126-164 (step order).
"""
import torch
import torch.nn.functional as F


def _bn(sd, name, y, train):
    return F.batch_norm(y, sd[name + ".running_mean"], sd[name + ".running_var"],
                        sd[name + ".weight"], sd[name + ".bias"], training=train,
                        momentum=0.1, eps=1e-5)


def _count(sd, names, train):
    if train:
        for n in names:
            sd[n + ".num_batches_tracked"] += 1


def _head(sd, h, train, keep):
    if "attention.conv.weight" in sd:
        a = torch.sigmoid(F.conv2d(h, sd["attention.conv.weight"], sd["attention.conv.bias"]))
        if keep is not None:
            keep["att"] = a
        h = h * a
    pooled = h.mean(dim=(2, 3))
    if keep is not None:
        keep["pooled"] = pooled
    z = F.linear(pooled, sd["projection.0.weight"], sd["projection.0.bias"])
    z = _bn(sd, "projection.1", z, train)
    _count(sd, ["projection.1"], train)
    return F.normalize(z, p=2, dim=1)


def small_forward(sd, x, train=True, masks=None, keep=None):
    """PhonemeNet.forward; keep (dict) collects y_l (conv outputs) and z_l (BN outputs, with
    retain_grad) for l = 1..6 so tests can compare intermediates and their gradients."""
    h = x
    layer = 0
    for blk in range(3):
        for ci, bi in ((0, 1), (3, 4)):
            layer += 1
            pre = f"conv_blocks.{blk}."
            y = F.conv2d(h, sd[pre + f"{ci}.weight"], sd[pre + f"{ci}.bias"], padding=1)
            z = _bn(sd, pre + str(bi), y, train)
            _count(sd, [pre + str(bi)], train)
            if keep is not None:
                keep[f"y{layer}"] = y
                if z.requires_grad:
                    z.retain_grad()
                keep[f"z{layer}"] = z
            h = F.relu(z)
        if blk < 2:
            h = F.max_pool2d(h, 2, 2)
        if train and masks is not None:
            h = h * masks[blk][:, :, None, None]
    return _head(sd, h, train, keep)


def deep_forward(sd, x, train=True, masks=None, keep=None):
    """PhonemeNetDeep.forward with ResidualBlocks (reference phoneme_cnn.py:146-304)."""
    h = F.conv2d(x, sd["init_conv.0.weight"], sd["init_conv.0.bias"], padding=3)
    h = F.relu(_bn(sd, "init_conv.1", h, train))
    _count(sd, ["init_conv.1"], train)
    h = F.max_pool2d(h, 3, 2, 1)
    i = 0
    while f"conv_blocks.{i}.conv1.weight" in sd:
        pre = f"conv_blocks.{i}."
        s = 1 if i == 0 else 2
        out = F.conv2d(h, sd[pre + "conv1.weight"], sd[pre + "conv1.bias"], stride=s, padding=1)
        out = F.relu(_bn(sd, pre + "bn1", out, train))
        if train and masks is not None:
            out = out * masks[i][:, :, None, None]
        out = F.conv2d(out, sd[pre + "conv2.weight"], sd[pre + "conv2.bias"], padding=1)
        out = _bn(sd, pre + "bn2", out, train)
        names = [pre + "bn1", pre + "bn2"]
        if pre + "shortcut.0.weight" in sd:
            sc = F.conv2d(h, sd[pre + "shortcut.0.weight"], sd[pre + "shortcut.0.bias"], stride=s)
            sc = _bn(sd, pre + "shortcut.1", sc, train)
            names.append(pre + "shortcut.1")
        else:
            sc = h
        _count(sd, names, train)
        h = F.relu(out + sc)
        if keep is not None:
            keep[f"block{i}"] = h
        i += 1
    return _head(sd, h, train, keep)


def forward(sd, x, train=True, masks=None, keep=None):
    fn = deep_forward if "init_conv.0.weight" in sd else small_forward
    return fn(sd, x, train, masks, keep)


def supcon(f, labels, temperature=0.07, base_temperature=0.07):
    """SupervisedContrastiveLoss, reduction='mean' (reference losses.py:41-86)."""
    b = f.shape[0]
    m = (labels.view(-1, 1) == labels.view(1, -1)).to(f.dtype)
    lm = 1.0 - torch.eye(b, dtype=f.dtype, device=f.device)
    m = m * lm
    logits = f @ f.T / temperature
    logits = logits - logits.max(dim=1, keepdim=True)[0].detach()
    log_prob = logits - torch.log((torch.exp(logits) * lm).sum(1, keepdim=True) + 1e-6)
    ms = m.sum(1)
    ms = torch.where(ms == 0, torch.ones_like(ms), ms)
    return (-(temperature / base_temperature) * (m * log_prob).sum(1) / ms).mean()


def param_names(sd):
    return [k for k in sd if not (k.endswith("running_mean") or k.endswith("running_var")
                                  or k.endswith("num_batches_tracked"))]


class CpuTrainer:
    """One ContrastiveTrainer step on the CPU: forward, SupCon, backward, Adam.step."""

    def __init__(self, sd, temperature=0.15, lr=3e-4, weight_decay=1e-4, dtype=torch.float32):
        self.sd = {k: (v.clone().to(dtype) if v.is_floating_point() else v.clone()) for k, v in sd.items()}
        self.names = param_names(self.sd)
        for k in self.names:
            self.sd[k].requires_grad_(True)
        self.opt = torch.optim.Adam([self.sd[k] for k in self.names], lr=lr, weight_decay=weight_decay)
        self.temperature = temperature

    def step(self, x, labels, masks=None):
        e = forward(self.sd, x, True, masks)
        loss = supcon(e, labels, self.temperature, 0.07)
        self.opt.zero_grad()
        loss.backward()
        self.opt.step()
        return loss.detach()
