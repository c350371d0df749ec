"""One rank of the data-parallel product path, run as a child process by tests/test_ddp_gpu.py.

Each scenario: the HIP model (libpcx) forward + SupCon + backward on this rank's shard of a golden
case, then ContrastiveTrainer._reduce_clip_step -- the trainer's own all-reduce (one flat
collective, or GradBucketer buckets launched behind the native backward) + optional device-side
clip + FusedAdam.step(flat_grads, grad_scale = 1/world) -- exactly the step order of the
reference's _train_epoch (src/training/trainer.py:143-152).  Writes parameters, Adam moments and
the loss of every scenario to <out_dir>/rank<r>.npz.

    RANK=r WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=p PCX_DIST_BACKEND=gloo \
        python tests/ddp_worker.py OUT_DIR
"""
import logging
import os
import sys
import tempfile

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

# (name, golden case, model config, bucketed, gradient_clip_val)
SCENARIOS = [
    ("small_flat", "cnn_small_T201", {"embedding_dim": 128, "use_attention": True, "dropout_rate": 0.1}, False, None),
    ("small_bucket_clip", "cnn_small_T201", {"embedding_dim": 128, "use_attention": True, "dropout_rate": 0.1},
     True, 0.05),
    ("deep_flat", "cnn_deep_T200", {"embedding_dim": 128, "use_attention": True, "dropout_rate": 0.2,
                                    "hidden_dims": [8, 16, 32, 64]}, False, None),
    ("deep_bucket", "cnn_deep_T200", {"embedding_dim": 128, "use_attention": True, "dropout_rate": 0.2,
                                      "hidden_dims": [8, 16, 32, 64]}, True, None),
]


def run(name, case, cfg, bucketed, clip, rank, world, out):
    from golden_util import model_case
    from phoneme_contrast_amd import distributed as ddp
    from phoneme_contrast_amd.losses import SupervisedContrastiveLoss
    from phoneme_contrast_amd.models import model_registry
    from phoneme_contrast_amd.optim import FusedAdam
    from phoneme_contrast_amd.trainer import ContrastiveTrainer

    c = model_case(case)
    kind = "phoneme_cnn_deep" if "deep" in case else "phoneme_cnn"
    m = model_registry.create(kind, cfg)
    state = {k: torch.tensor(v) for k, v in c["state0"].items()}
    if rank == 1:  # the broadcast must overwrite a diverged replica
        state = {k: v + 1.0 if v.is_floating_point() else v for k, v in state.items()}
    m.load_state_dict(state)
    m = m.cuda().train()
    ddp.broadcast_module(m)
    opt = FusedAdam(m.parameters(), lr=c["lr"], weight_decay=c["weight_decay"])
    loss_fn = SupervisedContrastiveLoss(temperature=c["temperature"])
    tmp = tempfile.mkdtemp(prefix=f"ddp_{name}_{rank}_")
    trainer = ContrastiveTrainer(model=m, train_loader=[], val_loader=None, loss_fn=loss_fn, optimizer=opt,
                                 scheduler=None, device=torch.device("cuda"),
                                 config={"gradient_clip_val": clip} if clip else {}, output_dir=tmp,
                                 logger=logging.getLogger("ddp_worker"))
    assert trainer.world_size == world
    bucketer = ddp.GradBucketer(m, bucket_bytes=1024) if bucketed else None
    B = c["x"].shape[0]
    lo, hi = ddp.shard(B, rank, world)
    m.set_dropout_masks([torch.tensor(k[lo:hi]) for k in c["steps"][0]["masks"]])
    x = torch.tensor(c["x"][lo:hi]).cuda()
    labels = torch.tensor(c["labels"][lo:hi]).cuda()
    loss = loss_fn(m(x), labels)
    opt.zero_grad()
    loss.backward()
    nb = len(bucketer.buckets(next(iter(m._plans.values())))) if bucketer else 1
    if not bucketer:  # this rank's own gradient, before the all-reduce
        out[f"{name}/local"] = opt.flat_grad_views()[0].cpu().numpy().copy()
    trainer._reduce_clip_step()
    torch.cuda.synchronize()
    st = opt._flat[0]
    out[f"{name}/loss"] = np.array([loss.item()])
    out[f"{name}/flat"] = st["flat"].cpu().numpy()
    out[f"{name}/m"] = st["m"].cpu().numpy()
    out[f"{name}/v"] = st["v"].cpu().numpy()
    out[f"{name}/nbuckets"] = np.array([nb])
    if bucketer:
        bucketer.detach()


def run_groups(rank, world, out):
    """FusedAdam with two parameter groups (different weight decay) behind the trainer: bucketed
    (GradBucketer.finish cuts the summed buffer per group; group 1 starts at an unaligned offset)
    and flat all-reduce must give bit-identical updates (finish() used to return one
    buffer for every group)."""
    from golden_util import model_case
    from phoneme_contrast_amd import distributed as ddp
    from phoneme_contrast_amd.losses import SupervisedContrastiveLoss
    from phoneme_contrast_amd.models import model_registry
    from phoneme_contrast_amd.optim import FusedAdam
    from phoneme_contrast_amd.trainer import ContrastiveTrainer

    c = model_case("cnn_small_T201")
    for name, bucketed in (("groups_flat", False), ("groups_bucket", True)):
        m = model_registry.create("phoneme_cnn", {"embedding_dim": 128, "use_attention": True, "dropout_rate": 0.1})
        m.load_state_dict({k: torch.tensor(v) for k, v in c["state0"].items()})
        m = m.cuda().train()
        ps = list(m.parameters())
        opt = FusedAdam([{"params": ps[:26]}, {"params": ps[26:], "weight_decay": 1e-3}], lr=c["lr"],
                        weight_decay=c["weight_decay"])
        loss_fn = SupervisedContrastiveLoss(temperature=c["temperature"])
        trainer = ContrastiveTrainer(model=m, train_loader=[], val_loader=None, loss_fn=loss_fn, optimizer=opt,
                                     scheduler=None, device=torch.device("cuda"), config={},
                                     output_dir=tempfile.mkdtemp(prefix=f"ddp_{name}_{rank}_"),
                                     logger=logging.getLogger("ddp_worker"))
        bucketer = ddp.GradBucketer(m, bucket_bytes=1024) if bucketed else None
        B = c["x"].shape[0]
        lo, hi = ddp.shard(B, rank, world)
        m.set_dropout_masks([torch.tensor(k[lo:hi]) for k in c["steps"][0]["masks"]])
        loss = loss_fn(m(torch.tensor(c["x"][lo:hi]).cuda()), torch.tensor(c["labels"][lo:hi]).cuda())
        opt.zero_grad()
        loss.backward()
        trainer._reduce_clip_step()
        torch.cuda.synchronize()
        for gi in range(2):
            st = opt._flat[gi]
            for key in ("flat", "m", "v"):
                out[f"{name}/{gi}/{key}"] = st[key].cpu().numpy()
        if bucketer:
            bucketer.detach()


def run_global(rank, world, out):
    """Global-batch SupCon (GlobalSupervisedContrastiveLoss): (a) the loss alone on this rank's rows
    of a seeded global embedding batch, reductions mean / none; (b) a cnn_small trainer step on the
    golden case's shard, whose gradients the trainer SUMS (grad_scale 1)."""
    from golden_util import model_case
    from phoneme_contrast_amd import distributed as ddp
    from phoneme_contrast_amd.losses import GlobalSupervisedContrastiveLoss
    from phoneme_contrast_amd.models import model_registry
    from phoneme_contrast_amd.optim import FusedAdam
    from phoneme_contrast_amd.trainer import ContrastiveTrainer

    g = torch.Generator().manual_seed(77)
    fg = torch.nn.functional.normalize(torch.randn(2 * 384, 128, generator=g), dim=1)
    lab = torch.randint(0, 40, (2 * 384,), generator=g)
    lo, hi = ddp.shard(fg.shape[0], rank, world)
    for red in ("mean", "none"):
        f = fg[lo:hi].clone().cuda().requires_grad_(True)
        loss = GlobalSupervisedContrastiveLoss(temperature=0.1, reduction=red)(f, lab[lo:hi].cuda())
        (loss.sum() if loss.dim() else loss).backward()
        out[f"gloss_{red}/loss"] = np.atleast_1d(loss.detach().cpu().numpy())
        out[f"gloss_{red}/grad"] = f.grad.cpu().numpy()

    c = model_case("cnn_small_T201")
    m = model_registry.create("phoneme_cnn", {"embedding_dim": 128, "use_attention": True, "dropout_rate": 0.1})
    m.load_state_dict({k: torch.tensor(v) for k, v in c["state0"].items()})
    m = m.cuda().train()
    opt = FusedAdam(m.parameters(), lr=c["lr"], weight_decay=c["weight_decay"])
    loss_fn = GlobalSupervisedContrastiveLoss(temperature=c["temperature"])
    tmp = tempfile.mkdtemp(prefix=f"ddp_global_{rank}_")
    trainer = ContrastiveTrainer(model=m, train_loader=[], val_loader=None, loss_fn=loss_fn, optimizer=opt,
                                 scheduler=None, device=torch.device("cuda"), config={}, output_dir=tmp,
                                 logger=logging.getLogger("ddp_worker"))
    B = c["x"].shape[0]
    lo, hi = ddp.shard(B, rank, world)
    m.set_dropout_masks([torch.tensor(k[lo:hi]) for k in c["steps"][0]["masks"]])
    loss = loss_fn(m(torch.tensor(c["x"][lo:hi]).cuda()), torch.tensor(c["labels"][lo:hi]).cuda())
    opt.zero_grad()
    loss.backward()
    out["small_global/local"] = opt.flat_grad_views()[0].cpu().numpy().copy()
    trainer._reduce_clip_step()
    torch.cuda.synchronize()
    out["small_global/loss"] = np.array([loss.item()])
    out["small_global/m"] = opt._flat[0]["m"].cpu().numpy()


def main():
    out_dir = sys.argv[1]
    from phoneme_contrast_amd import distributed as ddp
    rank, world, local = ddp.init_from_env(backend="gloo")
    torch.cuda.set_device(ddp.local_device_index(local, torch.cuda.device_count()))
    out = {}
    for sc in SCENARIOS:
        run(*sc, rank, world, out)
    run_groups(rank, world, out)
    run_global(rank, world, out)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **out)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()
    print(f"rank {rank}: ok", flush=True)


if __name__ == "__main__":
    main()
