"""GPU localisation aid (not collected by pytest): per-layer errors of the PhonemeNet forward
activations y1..y6 and BN-output gradients dz1..dz6 against the float64 torch-CPU port."""
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from golden_util import model_case  # noqa: E402
from oracle import torch_port as tp  # noqa: E402
from phoneme_contrast_amd.losses import SupervisedContrastiveLoss  # noqa: E402
from phoneme_contrast_amd.models import PhonemeNet  # noqa: E402


def main(name="cnn_small_T200", cfg=None):
    c = model_case(name)
    cfg = cfg or {"embedding_dim": 128, "use_attention": True, "dropout_rate": 0.1}
    sd = {k: torch.tensor(v).double() if v.dtype.kind == "f" else torch.tensor(v) for k, v in c["state0"].items()}
    for k in tp.param_names(sd):
        sd[k].requires_grad_(True)
    masks = [torch.tensor(k).double() for k in c["steps"][0]["masks"]]
    keep = {}
    x = torch.tensor(c["x"]).double()
    e = tp.forward(sd, x, True, masks, keep)
    loss = tp.supcon(e, torch.tensor(c["labels"]), c["temperature"], 0.07)
    de = torch.autograd.grad(loss, e, retain_graph=True)[0]
    loss.backward()

    m = PhonemeNet(cfg)
    m.load_state_dict({k: torch.tensor(v) for k, v in c["state0"].items()})
    m.cuda().train()
    m.set_dropout_masks([torch.tensor(k) for k in c["steps"][0]["masks"]])
    xg = x.float().cuda()
    params = tuple(m.parameters())
    emb, ws, plan, gm = m._native_forward(xg, params)
    torch.cuda.synchronize()
    print("emb err", (emb.cpu().double() - e.detach()).abs().max().item())
    for l in range(1, 7):
        ref = keep[f"y{l}"].detach()
        got = plan.region(ws, f"y{l}", ref.shape).cpu().double()
        print(f"y{l}", tuple(ref.shape), "err %.3e  max %.3e" % ((got - ref).abs().max().item(), ref.abs().max().item()))
    lg = SupervisedContrastiveLoss(c["temperature"])
    embg = emb.clone().requires_grad_(True)
    lossg = lg(embg, torch.tensor(c["labels"]).cuda())
    lossg.backward()
    print("loss", lossg.item(), loss.item(), "dE err", (embg.grad.cpu().double() - de).abs().max().item())
    grads = m._native_backward(plan, ws, xg, emb, embg.grad, params, gm)
    torch.cuda.synchronize()
    for l in range(6, 0, -1):
        ref = keep[f"z{l}"].grad
        got = plan.region(ws, f"dz{l}", ref.shape).cpu().double()
        err = (got - ref).abs()
        print(f"dz{l}", "err %.3e  max %.3e" % (err.max().item(), ref.abs().max().item()))
        if l in (2, 4):  # MaxPool2 follows: are the largest errors at near-tied 2x2 windows?
            r = torch.relu(keep[f"z{l}"].detach())
            Hp, Wp = r.shape[2] // 2, r.shape[3] // 2
            win = r[:, :, :2 * Hp, :2 * Wp].reshape(r.shape[0], r.shape[1], Hp, 2, Wp, 2)
            win = win.permute(0, 1, 2, 4, 3, 5).reshape(r.shape[0], r.shape[1], Hp, Wp, 4)
            top = win.topk(2, dim=-1).values
            gap = (top[..., 0] - top[..., 1])
            e2 = err[:, :, :2 * Hp, :2 * Wp].reshape(r.shape[0], r.shape[1], Hp, 2, Wp, 2).amax(dim=(3, 5))
            idx = e2.flatten().topk(5).indices
            print(f"   worst dz{l} windows: err", [f"{e2.flatten()[i].item():.2e}" for i in idx],
                  "top-2 gap", [f"{gap.flatten()[i].item():.2e}" for i in idx])
    for (k, p), g in zip(m.named_parameters(), grads):
        ref = sd[k].grad
        print(f"grad {k:32s} relerr %.3e  max %.3e" % ((g.cpu().double() - ref).abs().max().item() / (ref.abs().max().item() + 1e-30), ref.abs().max().item()))


if __name__ == "__main__":
    main(*sys.argv[1:2])
