"""Generate the golden parity fixtures under tests/golden/ from the REFERENCE implementation.

Test infrastructure only.  This script is run by hand in the build container, where the
read-only reference checkout lives at /root/reference; it imports the reference's own modules
(`src.models`, `src.training.losses`) and records their inputs and outputs as .npz data.
Nothing in the shipped package, in `bench.py` or in the `-m gpu` tests imports the reference:
they read only the .npz files written here.

    cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/tests/golden/make_golden.py

What is recorded (reference file:line of the code being pinned):
  supcon.npz      SupervisedContrastiveLoss / NTXentLoss forward + autograd dF
                  (src/training/losses.py:41-86, :101-151)
  cnn_small_*.npz PhonemeNet train steps: embeddings, loss, every parameter gradient,
                  state after two Adam(lr=3e-4, wd=1e-4) steps, and the Dropout2d masks the
                  reference drew (captured with forward hooks so the build can inject them)
                  (src/models/phoneme_cnn.py:10-126, scripts/train.py:128-133)
  cnn_small_eval.npz  eval-mode forward (running stats, no dropout) (phoneme_cnn.py:98-126)
  cnn_deep_*.npz  PhonemeNetDeep with reduced widths hidden_dims=[8,16,32,64] (full topology)
                  (src/models/phoneme_cnn.py:146-304)
"""
import os
import sys

import numpy as np

REF = os.environ.get("PCX_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from src.models import model_registry  # noqa: E402  (reference)
from src.training.losses import NTXentLoss, SupervisedContrastiveLoss  # noqa: E402

torch.set_num_threads(8)


def f32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def sampler_labels(b):
    # ContrastiveBatchSampler layout (samplers.py:96-113) after _prepare_batch's
    # repeat_interleave(V) (trainer.py:193-197): every class occupies 4 consecutive rows.
    return torch.arange(b // 4).repeat_interleave(4)


# ----------------------------------------------------------------------------- SupCon
def make_supcon():
    cases = {}
    g = torch.Generator().manual_seed(1234)

    def add(name, B, D, T, labels, reduction="mean", base_T=0.07, mask=None, kind="supcon"):
        feats = F.normalize(torch.randn(B, D, generator=g, dtype=torch.float32), dim=1)
        feats.requires_grad_(True)
        if kind == "supcon":
            fn = SupervisedContrastiveLoss(temperature=T, base_temperature=base_T, reduction=reduction)
            loss = fn(feats, labels, mask=mask)
        else:
            fn = NTXentLoss(temperature=T, reduction=reduction)
            loss = fn(feats, labels)
        (loss.sum() if loss.dim() else loss).backward()
        cases[f"{name}/features"] = f32(feats)
        cases[f"{name}/labels"] = labels.numpy().astype(np.int64)
        cases[f"{name}/loss"] = f32(loss).reshape(-1)
        cases[f"{name}/grad"] = f32(feats.grad)
        cases[f"{name}/meta"] = np.array([B, D, T, base_T], dtype=np.float64)
        cases[f"{name}/reduction"] = np.array(reduction)
        cases[f"{name}/kind"] = np.array(kind)
        if mask is not None:
            cases[f"{name}/mask"] = mask.numpy().astype(np.float32)

    add("b8_t05", 8, 128, 0.5, torch.tensor([0, 0, 1, 1, 2, 2, 3, 3]))
    add("b2_t015", 2, 64, 0.15, torch.tensor([3, 3]))
    add("b24_t015", 24, 128, 0.15, sampler_labels(24))
    add("b256_t007", 256, 128, 0.07, sampler_labels(256))
    add("b256_d64_t015", 256, 64, 0.15, sampler_labels(256))
    # singleton classes -> zero-positive rows still count in the mean (losses.py:73-76)
    lab = sampler_labels(64).clone()
    lab[::7] = 1000 + torch.arange(lab[::7].numel())
    add("b64_singletons", 64, 128, 0.15, lab)
    add("b24_sum", 24, 128, 0.15, sampler_labels(24), reduction="sum")
    add("b24_none", 24, 128, 0.15, sampler_labels(24), reduction="none")
    lab = torch.tensor([0, 0, 1, 1, 0, 2, 2, 1, 3, 3, 3, 0])
    add("b12_mask", 12, 64, 0.15, lab, mask=torch.eq(lab[:, None], lab[None, :]).float())
    add("b24_ntxent", 24, 128, 0.15, sampler_labels(24), kind="ntxent")
    add("b24_ntxent_sum", 24, 128, 0.5, sampler_labels(24), reduction="sum", kind="ntxent")
    np.savez_compressed(os.path.join(OUT, "supcon.npz"), **cases)


# ----------------------------------------------------------------------------- models
class MaskRecorder:
    """Forward hooks on every nn.Dropout2d: record the per-(sample, channel) keep-scale the
    reference drew (0 or 1/(1-p)); channels whose input is all zero are recorded as 0."""

    def __init__(self, model):
        self.masks = []
        self.handles = [m.register_forward_hook(self.hook) for m in model.modules()
                        if isinstance(m, nn.Dropout2d)]

    def hook(self, mod, inp, out):
        x = inp[0].detach()
        y = out.detach()
        if not mod.training or mod.p == 0.0:
            self.masks.append(torch.ones(x.shape[0], x.shape[1]))
            return
        xs = x.abs().sum(dim=(2, 3))
        ys = y.abs().sum(dim=(2, 3))
        m = torch.where(xs > 0, ys / xs.clamp_min(1e-30), torch.zeros_like(xs))
        keep = 1.0 / (1.0 - mod.p)
        m = torch.where(m > 0.5 * keep, torch.full_like(m, keep), torch.zeros_like(m))
        self.masks.append(m)

    def take(self):
        out, self.masks = self.masks, []
        return out


def train_steps(name, model_type, cfg, B, T, n_steps, seed_x, temp=0.15, lr=3e-4, wd=1e-4,
                store_state=True):
    torch.manual_seed(42)
    model = model_registry.create(model_type, cfg)
    model.train()
    rec = MaskRecorder(model)
    state0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
    opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=wd)
    loss_fn = SupervisedContrastiveLoss(temperature=temp)
    gx = torch.Generator().manual_seed(seed_x)
    x = torch.randn(B, 1, 40, T, generator=gx)
    labels = sampler_labels(B)
    out = {"x": f32(x), "labels": labels.numpy().astype(np.int64),
           "meta": np.array([B, T, temp, lr, wd], dtype=np.float64)}
    if store_state:
        for k, v in state0.items():
            out[f"state0/{k}"] = v.numpy()
    for step in range(n_steps):
        emb = model(x)
        masks = rec.take()
        loss = loss_fn(emb, labels)
        opt.zero_grad()
        loss.backward()
        out[f"step{step}/emb"] = f32(emb)
        out[f"step{step}/loss"] = f32(loss).reshape(1)
        for i, m in enumerate(masks):
            out[f"step{step}/mask{i}"] = m.numpy().astype(np.float32)
        if step == 0:
            for k, p in model.named_parameters():
                out[f"grad/{k}"] = f32(p.grad)
        opt.step()
    if n_steps > 1 or store_state:
        for k, v in model.state_dict().items():
            out[f"state_final/{k}"] = v.detach().numpy()
    # the same first step re-run by the reference in float64 with the recorded masks injected:
    # the fp64 truth that pins the float64 oracle tightly (fp32 runs can flip ReLU kinks)
    torch.manual_seed(42)
    m64 = model_registry.create(model_type, cfg).double()
    m64.load_state_dict({k: v.clone() for k, v in state0.items()})
    m64.train()
    queue = [torch.from_numpy(out[f"step0/mask{i}"]).double()
             for i in range(sum(1 for k in out if k.startswith("step0/mask")))]

    def inject(mod, inp):
        mk = queue.pop(0)
        return (inp[0] * mk[:, :, None, None],)

    for mod in m64.modules():
        if isinstance(mod, nn.Dropout2d):
            mod.p = 0.0
            mod.register_forward_pre_hook(inject)
    e64 = m64(x.double())
    l64 = loss_fn(e64, labels)
    l64.backward()
    out["f64/emb"] = f32(e64)
    out["f64/loss"] = l64.detach().numpy().astype(np.float64).reshape(1)
    for k, p in m64.named_parameters():
        out[f"f64/grad/{k}"] = f32(p.grad)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)
    return state0


def make_eval(state0):
    torch.manual_seed(42)
    model = model_registry.create("phoneme_cnn", {"embedding_dim": 128})
    model.load_state_dict(state0)
    # non-trivial running statistics so eval mode is actually exercised
    g = torch.Generator().manual_seed(7)
    for k, v in model.state_dict().items():
        if k.endswith("running_mean"):
            v.copy_(0.1 * torch.randn(v.shape, generator=g))
        elif k.endswith("running_var"):
            v.copy_(0.5 + torch.rand(v.shape, generator=g))
    model.eval()
    out = {}
    for k, v in model.state_dict().items():
        out[f"state/{k}"] = v.numpy()
    for B in (1, 4):
        x = torch.randn(B, 1, 40, 100, generator=g)
        with torch.no_grad():
            e = model(x)
        out[f"b{B}/x"] = f32(x)
        out[f"b{B}/emb"] = f32(e)
    np.savez_compressed(os.path.join(OUT, "cnn_small_eval.npz"), **out)


if __name__ == "__main__":
    make_supcon()
    small = {"in_channels": 1, "embedding_dim": 128, "use_attention": True, "dropout_rate": 0.1}
    st = train_steps("cnn_small_T200", "phoneme_cnn", small, B=8, T=200, n_steps=2, seed_x=1234)
    train_steps("cnn_small_T201", "phoneme_cnn", small, B=8, T=201, n_steps=1, seed_x=99,
                store_state=False)
    train_steps("cnn_small_noattn_d64", "phoneme_cnn",
                {"embedding_dim": 64, "use_attention": False, "dropout_rate": 0.1},
                B=16, T=50, n_steps=1, seed_x=5, temp=0.5)
    make_eval(st)
    deep = {"in_channels": 1, "embedding_dim": 128, "use_attention": True, "dropout_rate": 0.2,
            "hidden_dims": [8, 16, 32, 64], "use_residual": True}
    train_steps("cnn_deep_T200", "phoneme_cnn_deep", deep, B=8, T=200, n_steps=2, seed_x=4321)
    train_steps("cnn_deep_T201", "phoneme_cnn_deep", deep, B=8, T=201, n_steps=1, seed_x=77)
    for f in sorted(os.listdir(OUT)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(OUT, f)))
