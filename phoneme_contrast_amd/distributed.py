"""Data parallelism for the train step: one process per GPU, RCCL over xGMI.

The reference trains on one device (src/utils/device.py:39-42); this adds DDP-equivalent
semantics: every rank runs the full model on its own shard of the batch with its
own BatchNorm statistics and SupCon negatives, the gradients of the whole model are summed in ONE
flat all-reduce (1.2 MB for cnn_small: latency-bound, a single bucket), and the 1/world_size
average is folded into the Adam kernel (grad_scale).  Parameters and buffers are broadcast from
rank 0 once.  Backend "nccl" is RCCL on ROCm; "gloo" serves the CPU tests.
"""
import os

import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def init_from_env(backend=None):
    """Initialise the process group from torchrun's env (RANK, WORLD_SIZE, LOCAL_RANK,
    MASTER_ADDR/PORT).  Returns (rank, world_size, local_rank); no-op for a single process."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    if ws <= 1:
        return 0, 1, lr
    if backend is None:  # PCX_DIST_BACKEND=gloo rehearses N ranks on one GPU (tests only)
        backend = os.environ.get("PCX_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        torch.cuda.set_device(lr)
    if not dist.is_initialized():
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", lr)
        dist.init_process_group(backend=backend, **kw)
    return dist.get_rank(), dist.get_world_size(), lr


def shard(n_global: int, rank: int, world_size: int):
    """Row range [lo, hi) of rank `rank` when n_global rows are split into equal contiguous
    shards (keeps each class's consecutive rows together when n_global/world is a multiple of 4)."""
    per = n_global // world_size
    if per * world_size != n_global:
        raise ValueError(f"global batch {n_global} not divisible by world size {world_size}")
    return rank * per, (rank + 1) * per


@torch.no_grad()
def broadcast_module(module: torch.nn.Module, src: int = 0):
    """Make every rank start from rank `src`'s parameters and buffers."""
    if world()[1] == 1:
        return
    for t in list(module.parameters()) + list(module.buffers()):
        dist.broadcast(t.data, src)


def allreduce_flat(flat: torch.Tensor):
    """Sum one flat gradient bucket across ranks in place (a single collective per step)."""
    if world()[1] > 1:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    return flat
