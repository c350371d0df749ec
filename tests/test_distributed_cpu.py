"""Data-parallel path on CPU with the gloo backend, world_size 2 (the N>1 logic of bench.py and
the trainer): batch sharding, parameter broadcast, one flat all-reduce, 1/N averaging.
DDP-equivalent oracle: the float64 torch-CPU port run on each shard separately; the averaged
gradient must equal (1/N) * sum of per-shard gradients, and every rank must end up identical."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    from golden_util import model_case
    from oracle import torch_port as tp
    from phoneme_contrast_amd import distributed as ddp
    r, w, _ = ddp.init_from_env(backend="gloo")
    assert (r, w) == (rank, world)
    c = model_case("cnn_small_T201")
    sd = {k: torch.tensor(v).double() if v.dtype.kind == "f" else torch.tensor(v) for k, v in c["state0"].items()}
    if rank == 1:  # broadcast must overwrite a diverged replica
        for k in sd:
            if sd[k].is_floating_point():
                sd[k] += 1.0
    holder = torch.nn.Module()
    for i, (k, v) in enumerate(sd.items()):
        holder.register_buffer(f"b{i}", v)
    ddp.broadcast_module(holder)
    sd = {k: getattr(holder, f"b{i}") for i, k in enumerate(sd)}
    names = tp.param_names(sd)
    for k in names:
        sd[k].requires_grad_(True)
    x = torch.tensor(c["x"]).double()
    lab = torch.tensor(c["labels"])
    masks = [torch.tensor(m).double() for m in c["steps"][0]["masks"]]
    lo, hi = ddp.shard(x.shape[0], rank, world)
    e = tp.forward(sd, x[lo:hi], True, [m[lo:hi] for m in masks])
    loss = tp.supcon(e, lab[lo:hi], c["temperature"], 0.07)
    loss.backward()
    flat = torch.cat([sd[k].grad.reshape(-1) for k in names])
    ddp.allreduce_flat(flat)
    flat /= world
    out[rank] = flat.clone()
    torch.distributed.destroy_process_group()


def test_gloo_world2_flat_allreduce_matches_per_shard_average():
    from golden_util import model_case
    from oracle import torch_port as tp
    world = 2
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    assert torch.equal(out[0], out[1])
    # oracle: per-shard gradients computed in one process, averaged
    c = model_case("cnn_small_T201")
    x = torch.tensor(c["x"]).double()
    lab = torch.tensor(c["labels"])
    masks = [torch.tensor(m).double() for m in c["steps"][0]["masks"]]
    acc = None
    for r in range(world):
        sd = {k: torch.tensor(v).double() if v.dtype.kind == "f" else torch.tensor(v) for k, v in c["state0"].items()}
        names = tp.param_names(sd)
        for k in names:
            sd[k].requires_grad_(True)
        lo, hi = r * 4, (r + 1) * 4
        loss = tp.supcon(tp.forward(sd, x[lo:hi], True, [m[lo:hi] for m in masks]), lab[lo:hi], c["temperature"], 0.07)
        loss.backward()
        g = torch.cat([sd[k].grad.reshape(-1) for k in names])
        acc = g if acc is None else acc + g
    assert torch.allclose(out[0], acc / world, rtol=1e-10, atol=1e-12)


def test_shard_ranges():
    from phoneme_contrast_amd.distributed import shard
    assert [shard(32768, r, 8) for r in (0, 7)] == [(0, 4096), (28672, 32768)]
    with pytest.raises(ValueError):
        shard(10, 0, 3)


def _trainer_worker(rank, world, port, clip, out):
    """ContrastiveTrainer._reduce_clip_step itself on the generic (non-fused) path: a CPU model,
    torch.optim.Adam, gloo all-reduce of the per-rank gradients, torch's clip, step."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import logging
    import sys
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "tests")]
    from phoneme_contrast_amd import distributed as ddp
    from phoneme_contrast_amd.trainer import ContrastiveTrainer
    ddp.init_from_env(backend="gloo")
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Tanh(), torch.nn.Linear(5, 3))
    if rank == 1:
        with torch.no_grad():
            for p in model.parameters():
                p.add_(1.0)
    ddp.broadcast_module(model)
    opt = torch.optim.Adam(model.parameters(), lr=1e-2, weight_decay=1e-4)
    tr = ContrastiveTrainer(model, [], None, None, opt, None, torch.device("cpu"),
                            {"gradient_clip_val": clip} if clip else {}, tempfile.mkdtemp(),
                            logging.getLogger("t"))
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(8, 6, generator=g)
    opt.zero_grad()
    model(x).pow(2).sum().backward()
    tr._reduce_clip_step()
    out[(clip, rank)] = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("clip", [None, 0.5])
def test_gloo_world2_trainer_reduce_clip_step_generic_path(clip):
    world = 2
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    mp.start_processes(_trainer_worker, args=(world, _free_port(), clip, out), nprocs=world, join=True,
                       start_method="spawn")
    assert torch.equal(out[(clip, 0)], out[(clip, 1)])
    # single process: average of the two ranks' gradients, torch clip, one Adam step
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.Tanh(), torch.nn.Linear(5, 3))
    opt = torch.optim.Adam(model.parameters(), lr=1e-2, weight_decay=1e-4)
    grads = []
    for r in range(world):
        model.zero_grad()
        x = torch.randn(8, 6, generator=torch.Generator().manual_seed(100 + r))
        model(x).pow(2).sum().backward()
        grads.append([p.grad.clone() for p in model.parameters()])
    for p, *gs in zip(model.parameters(), *grads):
        p.grad = sum(gs) / world
    if clip:
        total = torch.nn.utils.clip_grad_norm_(model.parameters(), clip)
        assert total > clip  # clipping is live
    opt.step()
    ref = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    assert torch.allclose(out[(clip, 0)], ref, rtol=1e-6, atol=1e-7)
