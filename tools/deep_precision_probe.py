"""Analysis aid: conditioning of cnn_deep's block-3 weight gradients at B = 4096 (why float32
implementations disagree with float64 there).  Runs the float64 restatement on the GPU with the
block intermediates kept, then evaluates dW = conv2d_weight(x, dy) of block 3 conv2 in float64, in
torch float32 and in float32 with dy perturbed by one float32 rounding, and prints the condition
number sum|dy x| / |dW| per output element.

    python tools/deep_precision_probe.py [B]
"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
from oracle import torch_port as tp  # noqa: E402
from phoneme_contrast_amd.models import PhonemeNetDeep  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
torch.manual_seed(42)
m = PhonemeNetDeep({"embedding_dim": 128, "use_attention": True, "dropout_rate": 0.2, "hidden_dims": [64, 128, 256, 512]})
sd = {k: (v.double() if v.is_floating_point() else v).cuda() for k, v in m.state_dict().items()}
g = torch.Generator().manual_seed(4321)
x = torch.randn(B, 1, 40, 200, generator=g)
labels = torch.arange(B // 4).repeat_interleave(4).cuda()
masks = [((torch.rand(B, c, generator=g) >= 0.1).double() / 0.9).cuda() for c in (64, 128, 256, 512)]

# block-3 conv2: capture its input and the gradient w.r.t. its output with hooks on F.conv2d
cap = {}
orig = F.conv2d


def conv_hook(inp, w, b=None, stride=1, padding=0, *a, **k):
    out = orig(inp, w, b, stride, padding, *a, **k)
    if w is sd["conv_blocks.3.conv2.weight"]:
        cap["x"] = inp.detach()
        out.register_hook(lambda gr: cap.__setitem__("dy", gr.detach()))
    return out


F.conv2d = conv_hook
params = tp.param_names(sd)
for k in params:
    sd[k].requires_grad_(True)
e = tp.forward(sd, x.double().cuda(), True, masks)
loss = tp.supcon(e, labels, 0.15, 0.07)
loss.backward()
F.conv2d = orig
xin, dy = cap["x"], cap["dy"]
w = sd["conv_blocks.3.conv2.weight"]
ref = sd["conv_blocks.3.conv2.weight"].grad.detach()
gw64 = torch.nn.grad.conv2d_weight(xin, w.shape, dy, padding=1)
print("f64 dW recomputed vs autograd:", float((gw64 - ref).abs().max() / ref.abs().max()))
absum = torch.nn.grad.conv2d_weight(xin.abs(), w.shape, dy.abs(), padding=1)
cond = (absum / ref.abs().clamp(min=1e-300))
print("max|dW| %.3e  max sum|dy x| %.3e  median cond %.3e  cond at argmax|dW| %.3e" % (
    float(ref.abs().max()), float(absum.max()), float(cond.median()), float(cond.flatten()[ref.abs().argmax()])))
print("per-channel |sum dy| / sum|dy|: max %.3e" % float((dy.sum((0, 2, 3)).abs() / dy.abs().sum((0, 2, 3))).max()))
print("x mean / std (channels, median): %.3f" % float((xin.mean((0, 2, 3)) / xin.std((0, 2, 3))).median()))
with torch.backends.cudnn.flags(enabled=False):
    gw32 = torch.nn.grad.conv2d_weight(xin.float(), w.shape, dy.float(), padding=1).double()
print("torch f32 dW (exact f64 operands rounded once):", float((gw32 - ref).abs().max() / ref.abs().max()))
dyr = dy.float().double()
print("f64 dW on f32-rounded dy:", float((torch.nn.grad.conv2d_weight(xin, w.shape, dyr, padding=1) - ref).abs().max()
                                          / ref.abs().max()))
# a per-channel offset of dy of one float32 ulp of its mean |dy| (an inexact BN-backward mean)
off = dy.abs().mean((0, 2, 3), keepdim=True) * 2.0 ** -24
print("f64 dW with dy + 1-ulp channel offset:", float((torch.nn.grad.conv2d_weight(xin, w.shape, dy + off, padding=1)
                                                      - ref).abs().max() / ref.abs().max()))
