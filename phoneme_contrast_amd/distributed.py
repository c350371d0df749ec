"""Data parallelism for the train step: one process per GPU, RCCL over xGMI.

The reference trains on one device (src/utils/device.py:39-42); this adds DDP-equivalent
semantics: every rank runs the full model on its own shard of the batch with its
own BatchNorm statistics and SupCon negatives, the gradients of the whole model are summed by
all-reduce and the 1/world_size average is folded into the Adam kernel (grad_scale).  The sum is
either ONE flat all-reduce after the backward (cnn_small: 1.2 MB, latency-bound) or, with a
GradBucketer, a few buckets launched on a side stream as soon as the native backward has written
them (events recorded inside pcx_net_backward), so they overlap the remaining backward layers
(cnn_deep: 19.9 MB).  Parameters and buffers are broadcast from rank 0 once.  Backend "nccl" is
RCCL on ROCm; "gloo" serves the CPU tests and the N-ranks-on-one-GPU rehearsal.
"""
import ctypes
import os
import weakref

import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def init_from_env(backend=None):
    """Initialise the process group from torchrun's env (RANK, WORLD_SIZE, LOCAL_RANK,
    MASTER_ADDR/PORT).  Returns (rank, world_size, local_rank); no-op for a single process unless
    PCX_DIST_FORCE_INIT=1 (a world-1 group: runs the RCCL bucket path on a one-GPU box, where two
    RCCL ranks cannot share the device)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    if ws <= 1 and os.environ.get("PCX_DIST_FORCE_INIT") != "1":
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


@torch.no_grad()
def broadcast_buffers(module: torch.nn.Module, src: int = 0):
    """Rank `src`'s buffers (BatchNorm running statistics) on every rank."""
    if world()[1] == 1:
        return
    for t in module.buffers():
        dist.broadcast(t.data, src)


def is_distributed() -> bool:
    """A process group is up (any world size, including a forced world-1 group)."""
    return dist.is_available() and dist.is_initialized()


def allreduce_flat(flat: torch.Tensor):
    """Sum one flat gradient bucket across ranks in place (a single collective per step)."""
    if world()[1] > 1:
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
    return flat


def local_device_index(local_rank: int, n_devices: int) -> int:
    """GPU of a local rank: LOCAL_RANK on a full node; N ranks rehearsed on fewer GPUs
    (PCX_DIST_BACKEND=gloo on a one-GPU box) share them round-robin."""
    return local_rank % max(1, n_devices)


def covers(optimizer, module: torch.nn.Module) -> bool:
    """True when the optimizer's groups hold exactly the module's parameters, in order (so its
    flat gradient buffers ARE the module's gradients)."""
    ps = [p for g in optimizer.param_groups for p in g["params"]]
    ms = list(module.parameters())
    return len(ps) == len(ms) and all(a is b for a, b in zip(ps, ms))


@torch.no_grad()
def clip_flat_(flats, max_norm: float, scale: float = 1.0):
    """torch.nn.utils.clip_grad_norm_ on gradients held as flat buffers that still carry a factor
    1/scale (the rank sum before the 1/world average): norm = scale * ||flats||, and every buffer
    is multiplied in place by min(1, max_norm / (norm + 1e-6)).  Stays on the device."""
    total = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(f) for f in flats])) * scale
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    for f in flats:
        f.mul_(coef)
    return total


class GradBucketer:
    """All-reduce of the flat gradient in buckets that overlap the native backward.

    Bucket boundaries are backward stages of the plan (pcx_net_grad_stages): the last parameters
    (projection, attention, last block) finish first.  `bucket_bytes` is the target size: stages
    are merged from the end until a bucket reaches it.  The model calls `launch(plan, flat)` right
    after enqueueing its backward: for every bucket a side stream waits on the bucket's event and
    the collective is enqueued there (async), so bucket k is summed while the layers below it are
    still back-propagating.  `finish()` makes the current stream wait for all of them and returns
    [flat] for FusedAdam.step(flat_grads=..., grad_scale=1/world).  Sums are bit-identical to one
    flat all-reduce of the same buffer only up to the collective's own reduction order."""

    def __init__(self, model: torch.nn.Module, bucket_bytes: int = 4 << 20):
        self.model = model
        self.bucket_bytes = int(bucket_bytes)
        self.sizes = [p.numel() for p in model.parameters()]
        self.offsets = [0]
        for n in self.sizes:
            self.offsets.append(self.offsets[-1] + n)
        self._plans = weakref.WeakKeyDictionary()  # plan -> bucket first-parameter indices
        self._works = []
        self._flat = None
        self._stream = None
        model._grad_bucketer = self

    def detach(self):
        if getattr(self.model, "_grad_bucketer", None) is self:
            self.model._grad_bucketer = None

    def _configure(self, plan):
        from . import _lib
        key = plan
        firsts = self._plans.get(key)
        if firsts is not None:
            return firsts
        lib = _lib.lib()
        n = lib.pcx_net_grad_stages(plan.handle, None, 0)
        arr = (ctypes.c_int * max(1, n))()
        lib.pcx_net_grad_stages(plan.handle, arr, n)
        stages = [arr[i] for i in range(n)]
        if not stages or stages[-1] != 0:
            stages.append(0)
        firsts, hi = [], len(self.sizes)
        for st in stages:  # merge stages from the end until a bucket reaches bucket_bytes
            if 4 * (self.offsets[hi] - self.offsets[st]) >= self.bucket_bytes or st == 0:
                firsts.append(st)
                hi = st
        buf = (ctypes.c_int * len(firsts))(*firsts)
        _lib.check(lib.pcx_net_grad_buckets(plan.handle, len(firsts), buf), "pcx_net_grad_buckets")
        self._plans[key] = firsts
        return firsts

    def buckets(self, plan):
        """Element ranges [lo, hi) of the flat gradient, in launch order."""
        firsts = self._configure(plan)
        out, hi = [], len(self.sizes)
        for f in firsts:
            out.append((self.offsets[f], self.offsets[hi]))
            hi = f
        return out

    def prepare(self, plan):
        """Called before the native backward (installs the plan's bucket events)."""
        self._configure(plan)

    def launch(self, plan, flat: torch.Tensor):
        from . import _lib
        if not is_distributed():
            return
        if self._stream is None or self._stream.device != flat.device:
            self._stream = torch.cuda.Stream(device=flat.device)
        lib = _lib.lib()
        self._works = []
        for k, (lo, hi) in enumerate(self.buckets(plan)):
            _lib.check(lib.pcx_net_bucket_wait(plan.handle, k, ctypes.c_void_p(self._stream.cuda_stream)),
                       "pcx_net_bucket_wait")
            with torch.cuda.stream(self._stream):
                self._works.append(dist.all_reduce(flat[lo:hi], op=dist.ReduceOp.SUM, async_op=True))
        self._flat = flat

    def pending(self) -> bool:
        return self._flat is not None

    def finish(self, group_sizes=None):
        """Wait (on the current stream) for every bucket of the last backward.  Returns the summed
        gradient as one tensor per optimizer parameter group: `group_sizes` (element counts of the
        groups, in parameter order; default one group) cuts the flat buffer into consecutive
        slices, and a slice that does not start 16-byte aligned (pcx_adam_step's vector loads) is
        returned as an aligned copy."""
        flat = self._flat
        if flat is None:
            return None
        for w in self._works:
            w.wait()
        torch.cuda.current_stream(flat.device).wait_stream(self._stream)
        self._works, self._flat = [], None
        if group_sizes is None:
            return [flat]
        if sum(group_sizes) != flat.numel():
            raise ValueError(f"parameter groups hold {sum(group_sizes)} elements, the gradient {flat.numel()}")
        out, off = [], 0
        for n in group_sizes:
            g = flat[off:off + n]
            out.append(g if g.data_ptr() % 16 == 0 else g.clone())
            off += n
        return out
