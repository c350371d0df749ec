"""Analysis aid: weight-gradient engines at large K against float64.

(1) pcx_conv2d mode 2 (general engine, convg.hip) at cnn_deep block-3 shapes, B = 4096, vs float64
    torch.nn.grad.conv2d_weight on the same float32 operands.
(2) cnn_deep full model at B in {512, 1024, 2048, 4096}: error of every weight gradient vs the float64
    restatement (to see whether an error grows with B).

    python tools/wgrad_probe.py [1|2]
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def conv2d_wgrad(B, cin, cout, IH, IW, k, s, p):
    from phoneme_contrast_amd import _lib
    lib = _lib.lib()
    g = torch.Generator(device="cuda").manual_seed(B + cin)
    OH, OW = (IH + 2 * p - k) // s + 1, (IW + 2 * p - k) // s + 1
    x = torch.relu(torch.randn(B, cin, IH, IW, device="cuda", generator=g))
    dy = torch.randn(B, cout, OH, OW, device="cuda", generator=g)
    dy -= dy.mean((0, 2, 3), keepdim=True)  # BN-backward-like: zero mean per channel
    out = torch.empty(cout, cin, k, k, device="cuda")
    nb = lib.pcx_conv2d_workspace_bytes(2, 0, B, cin, cout, OH, OW, k)
    ws = torch.empty(max(nb, 4) // 4 + 1, device="cuda")
    _lib.check(lib.pcx_conv2d(2, 0, B, cin, cout, IH, IW, OH, OW, k, s, p, _lib.ptr(x), None, _lib.ptr(dy),
                              _lib.ptr(out), 0, _lib.ptr(ws), ws.numel() * 4,
                              ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "pcx_conv2d")
    ref = torch.nn.grad.conv2d_weight(x.double(), (cout, cin, k, k), dy.double(), stride=s, padding=p)
    err = float((out.double() - ref).abs().max() / ref.abs().max())
    print(f"convg wgrad B={B} {cin}->{cout} {IH}x{IW} k{k} s{s}: rel err {err:.3e}", flush=True)


def model_sweep():
    from oracle import torch_port as tp
    from phoneme_contrast_amd.losses import SupervisedContrastiveLoss
    from phoneme_contrast_amd.models import PhonemeNetDeep
    for B in (512, 1024, 2048, 4096):
        torch.manual_seed(42)
        m = PhonemeNetDeep({"embedding_dim": 128, "use_attention": True, "dropout_rate": 0.2,
                            "hidden_dims": [64, 128, 256, 512]})
        sd = {k: (v.double() if v.is_floating_point() else v).cuda() for k, v in m.state_dict().items()}
        m = m.cuda().train()
        gen = torch.Generator().manual_seed(4321)
        x = torch.randn(B, 1, 40, 200, generator=gen)
        labels = torch.arange(B // 4).repeat_interleave(4)
        masks = [(torch.rand(B, c, generator=gen) >= 0.1).float() / 0.9 for c in (64, 128, 256, 512)]
        m.set_dropout_masks(masks)
        loss = SupervisedContrastiveLoss(temperature=0.15)(m(x.cuda()), labels.cuda())
        loss.backward()
        got = {k: p.grad.double() for k, p in m.named_parameters()}
        del m
        params = tp.param_names(sd)
        for k in params:
            sd[k].requires_grad_(True)
        e = tp.forward(sd, x.double().cuda(), True, [k.double().cuda() for k in masks])
        tp.supcon(e, labels.cuda(), 0.15, 0.07).backward()
        errs = {k: float((got[k] - sd[k].grad).abs().max() / sd[k].grad.abs().max()) for k in params
                if k.endswith("weight") and ("conv" in k or "shortcut" in k)}
        top = sorted(errs.items(), key=lambda kv: -kv[1])[:6]
        print(f"B={B}: " + ", ".join(f"{k} {v:.2e}" for k, v in top), flush=True)
        del sd, e
        torch.cuda.empty_cache()


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "12"
    if "1" in which:
        for shp in [(4096, 256, 512, 5, 25, 3, 2, 1), (4096, 256, 512, 5, 25, 1, 2, 0), (4096, 512, 512, 3, 13, 3, 1, 1),
                    (4096, 128, 256, 10, 50, 3, 2, 1)]:
            conv2d_wgrad(*shp)
    if "2" in which:
        model_sweep()
