#!/usr/bin/env python
"""Benchmark of the north-star hot path: one contrastive train step of cnn_small at batch 4096
per GPU (reference: ContrastiveTrainer._train_epoch, src/training/trainer.py:126-164), i.e.
PhonemeNet forward + SupCon + backward + gradient all-reduce (N > 1) + Adam, on synthetic MFCC
tensors [B, 1, 40, 200].

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Rank 0 prints ONE JSON line.  `value` = MFCC samples processed by all ranks / wall time of the K
timed steps (max over ranks), inputs resident in HBM.  `roofline` is for the dominant kernel,
timed live with HIP events on its stream inside the timed region; `cpu_baseline` is the
float32 torch-CPU port of the reference step (oracle/torch_port.py) on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from phoneme_contrast_amd.costs import (BF16_PEAK_TFLOPS, DEEP_DIMS, FP32_PEAK_TFLOPS, HBM_PEAK_GBS,  # noqa: E402
                                        deep_executed_fraction, deep_kernel_costs, deep_step_cost,
                                        executed_fraction, executed_step_flops, kernel_costs, step_cost)

METRIC = "MFCC-samples/sec per train step (cnn_small, batch 4096) at 1/2/4/8 MI355X"


def sig(x, n=4):
    """x to n significant digits (a contended or tiny launch must not round to 0)."""
    return float(f"{x:.{n}g}")


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ----------------------------------------------------------------------------- CPU baseline
def cpu_model_name():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_leg(B, T, threads, min_s, min_steps, max_steps=200):
    """One timed leg of the float32 torch-CPU port of the reference train step: 1 warm-up step,
    then steps until min_s seconds and min_steps steps have passed."""
    from oracle import torch_port as tp
    from phoneme_contrast_amd.models import PhonemeNet
    torch.set_num_threads(threads)
    torch.manual_seed(42)
    sd = {k: v.clone() for k, v in PhonemeNet({"embedding_dim": 128, "dropout_rate": 0.1}).state_dict().items()}
    tr = tp.CpuTrainer(sd, temperature=0.15)
    g = torch.Generator().manual_seed(1234)
    x = torch.randn(B, 1, 40, T, generator=g)
    labels = torch.arange(B // 4).repeat_interleave(4)
    masks = [(torch.rand(B, c, generator=g) >= 0.1).float() / 0.9 for c in (32, 64, 128)]
    tw = time.perf_counter()
    tr.step(x, labels, masks)  # warm-up
    log(f"cpu baseline B={B} threads={threads}: warm-up step {time.perf_counter() - tw:.1f}s")
    n, t0 = 0, time.perf_counter()
    while True:
        tr.step(x, labels, masks)
        n += 1
        el = time.perf_counter() - t0
        if B >= 1024:
            log(f"cpu baseline B={B}: step {n} at {el:.1f}s")
        if (el >= min_s and n >= min_steps) or n >= max_steps:
            break
    return {"B": B, "threads": threads, "steps": n, "seconds": round(el, 2), "s_per_step": round(el / n, 3),
            "samples_per_s": round(B * n / el, 2)}


def cpu_baseline(full=False, quick=False, T=200):
    """The reference step on the host cores (the reference itself cannot travel to the GPU box):
    the float32 torch-CPU restatement (oracle/torch_port.py, pinned to the reference's own step
    within 10 %: profiles/cpu_port_vs_reference.json) at cores - 2 threads, the reference's rule
    (src/utils/device.py:58-61).  Legs: the headline batch B = 4096 (1 warm-up + 2 timed steps:
    the reported value, the same workload as the GPU number) and the reference's real train batch
    B = 24 (6 classes x 2 clips x 2 views, ~6 s); `full` adds both at all host threads, `quick`
    drops the B = 4096 leg.  The host is shared with other jobs of the GPU box, so legs vary by
    ~20 % between runs (round-3 B = 24 runs: 475-592 samples/s)."""
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 2)
    allc = max(1, min(share, os.cpu_count() or share))
    rule = max(1, allc - 2)
    legs = []
    if not quick:
        legs.append(_cpu_leg(4096, T, rule, 0.0, 2, 2))
    legs.append(_cpu_leg(24, T, rule, 6.0, 3))
    if full:
        if not quick:
            legs.append(_cpu_leg(4096, T, allc, 0.0, 2, 2))
        legs.append(_cpu_leg(24, T, allc, 6.0, 3))
    main = legs[0]
    what = ("the headline batch B=4096" if main["B"] == 4096 else "the reference's real batch B=24")
    return {"value": main["samples_per_s"], "unit": "samples/s", "cores": main["threads"], "kind": "port",
            "cpu_model": cpu_model_name(), "host_threads_available": allc,
            "sample": f"cnn_small train step (fwd+SupCon+bwd+Adam) at {what}, T={T}: {main['steps']} timed steps "
                      f"(after 1 warm-up) in {main['seconds']}s on cores-2 = {main['threads']} threads (reference "
                      "rule, src/utils/device.py:58-61); float32 torch-CPU restatement oracle/torch_port.py; "
                      "host shared with other jobs (legs vary ~20% run to run)", "legs": legs}


def measure_peaks(dev):
    """Achievable peaks on this box (report against vendor and measured): HBM by a 2 GiB
    float4 streaming copy (libpcx pcx_stream_copy: 16-byte nontemporal loads / stores, the copy the
    MI355X guide measures at ~6.3 TB/s; torch's copy_ reached ~4.9 TB/s, which understated the roof of
    an HBM-bound kernel), fp32 matrix rate by an 8192^3 torch.mm (rocBLAS / hipBLASLt fp32 GEMM on the
    MFMA).  Timed with HIP events on the current stream after a warm-up; ~1 s in total."""
    from phoneme_contrast_amd import _lib
    n = 1 << 29  # floats: 2 GiB per buffer
    a = torch.empty(n, device=dev)
    b = torch.empty(n, device=dev)
    so = _lib.lib()
    st = _lib.stream_of(a)

    def copy():
        _lib.check(so.pcx_stream_copy(_lib.ptr(a), _lib.ptr(b), 4 * n, st), "pcx_stream_copy")

    copy()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        copy()
    e1.record()
    torch.cuda.synchronize()
    hbm = 5 * 2 * 4 * n / (e0.elapsed_time(e1) / 1000.0) / 1e9
    e0.record()
    for _ in range(5):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    hbm_torch = 5 * 2 * 4 * n / (e0.elapsed_time(e1) / 1000.0) / 1e9
    del a, b
    m = 8192
    x = torch.randn(m, m, device=dev)
    y = torch.randn(m, m, device=dev)
    torch.mm(x, y)
    e0.record()
    for _ in range(5):
        torch.mm(x, y)
    e1.record()
    torch.cuda.synchronize()
    gemm = 5 * 2 * m ** 3 / (e0.elapsed_time(e1) / 1000.0) / 1e12
    return {"hbm_copy_GBps": round(hbm, 1), "hbm_torch_copy_GBps": round(hbm_torch, 1),
            "fp32_gemm_TFLOPs": round(gemm, 1),
            "note": "measured on this GPU: 2 GiB float4 streaming copy (pcx_stream_copy; read + write bytes), "
                    "torch copy_ beside it; torch.mm fp32 8192^3"}


def load_pmc(model, precision, label):
    """HBM bytes per launch of `label` in the (model, precision) workload from the committed
    rocprofv3 --pmc summary (profiles/pmc_traffic.json, keyed "<model>/<precision>"), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(f"{model}/{precision}", {}).get(label, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


# ----------------------------------------------------------------------------- N-GPU launch
def relaunch(n):
    """`--gpus N > 1` without torch.distributed.run's environment: start the N ranks as children under
    torch.distributed.run on this node (127.0.0.1, a free port) and return its exit code.  Runs before
    anything touches the GPU; the parent never measures, so an N-GPU request cannot print a 1-rank line."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    log(f"bench: --gpus {n} without WORLD_SIZE: launching {n} ranks under torch.distributed.run")
    return subprocess.run(cmd).returncode


def launch_check(args):
    """--launch-check: the launcher path alone (no model, no GPU): every rank joins the process group
    and rank 0 prints the ranks it saw (tests/test_bench_launch.py runs it on CPU with gloo)."""
    from phoneme_contrast_amd import distributed as ddp
    rank, world, _ = ddp.init_from_env(backend="gloo")
    seen = torch.distributed.get_world_size() if ddp.is_distributed() else 1
    if ddp.is_distributed():
        t = torch.ones(1)
        torch.distributed.all_reduce(t)
        seen = int(t.item())
    if rank == 0:
        print(json.dumps({"n_gpus": world, "dist_world_size": seen, "requested_gpus": args.gpus}), flush=True)
    if ddp.is_distributed():
        torch.distributed.destroy_process_group()
    return 0 if world == args.gpus == seen else 1


# ----------------------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096, help="per-GPU batch (views)")
    ap.add_argument("--T", type=int, default=200)
    ap.add_argument("--model", choices=["cnn_small", "cnn_deep"], default="cnn_small",
                    help="cnn_small is the north-star workload; cnn_deep is reported as a side line")
    ap.add_argument("--precision", choices=["fp32", "bf16"], default="fp32",
                    help="cnn_deep conv operand precision (bf16: float32 accumulation, float32 elsewhere)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-full", action="store_true", help="also time the CPU baseline legs at all host threads")
    ap.add_argument("--cpu-quick", action="store_true", help="CPU baseline at B=24 only (skip the B=4096 leg)")
    ap.add_argument("--bucket-mb", type=float, default=None,
                    help="N > 1: gradient all-reduce bucket size (default 0.5 MB cnn_small, 4 MB cnn_deep)")
    ap.add_argument("--global-supcon", action="store_true",
                    help="N > 1: SupCon over the global batch (embedding all-gather, sharded anchor rows)")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--table-steps", type=int, default=5,
                    help="untimed steps with every kernel event-timed (the per-kernel table)")
    ap.add_argument("--no-peaks", action="store_true", help="skip the measured-peak probes")
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and env_world is None:
        sys.exit(relaunch(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        log(f"error: --gpus {args.gpus} but WORLD_SIZE={env_world}: refusing to report a mismatched line")
        sys.exit(2)
    if args.launch_check:
        sys.exit(launch_check(args))

    from phoneme_contrast_amd import distributed as ddp
    from phoneme_contrast_amd.losses import GlobalSupervisedContrastiveLoss, SupervisedContrastiveLoss
    from phoneme_contrast_amd.models import model_registry
    from phoneme_contrast_amd.optim import FusedAdam

    rank, world, local = ddp.init_from_env()
    local = local % max(1, torch.cuda.device_count())  # == LOCAL_RANK on a full node
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    B, F, T, D = args.batch, 40, args.T, 128

    torch.manual_seed(42)
    deep = args.model == "cnn_deep"
    if deep:
        model = model_registry.create("phoneme_cnn_deep", {"in_channels": 1, "embedding_dim": D,
                                                           "use_attention": True, "dropout_rate": 0.2,
                                                           "hidden_dims": DEEP_DIMS,
                                                           "precision": args.precision})
    else:
        model = model_registry.create("phoneme_cnn", {"in_channels": 1, "embedding_dim": D,
                                                      "use_attention": True, "dropout_rate": 0.1})
    model = model.to(dev).train()
    ddp.broadcast_module(model)
    opt = FusedAdam(model.parameters(), lr=3e-4, weight_decay=1e-4)
    bucketer = None
    if ddp.is_distributed():  # buckets all-reduced on a side stream behind the native backward
        mb = args.bucket_mb if args.bucket_mb is not None else (4.0 if deep else 0.5)
        bucketer = ddp.GradBucketer(model, bucket_bytes=int(mb * (1 << 20)))
    loss_fn = (GlobalSupervisedContrastiveLoss if args.global_supcon else SupervisedContrastiveLoss)(temperature=0.15)
    gscale = 1.0 if args.global_supcon else 1.0 / world
    g = torch.Generator().manual_seed(1234 + rank)
    x = torch.randn(B, 1, F, T, generator=g).to(dev)
    labels = (torch.arange(B // 4).repeat_interleave(4) + rank * (B // 4)).to(dev)

    def step():
        e = model(x)
        loss = loss_fn(e, labels)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        if bucketer is not None:
            opt.step(flat_grads=bucketer.finish(), grad_scale=gscale)
        else:
            opt.step()
        return loss

    for _ in range(args.warmup):
        loss = step()
    torch.cuda.synchronize()
    log(f"rank {rank}: warm-up done, loss {loss.item():.4f}")

    bf16 = deep and args.precision == "bf16"
    costs = deep_kernel_costs(B, F, T, bf16, D) if deep else kernel_costs(B, F, T, D)
    timing = not args.no_kernel_timing
    table, tsteps, dom = {}, 0, None
    if timing:
        # per-kernel table: a few untimed steps with every launch event-timed; the timed region then
        # records the dominant costed kernel alone (one event pair per launch of it, not ~60 per step)
        tsteps = max(1, min(args.steps, args.table_steps))
        model.kernel_profile(True)
        for _ in range(tsteps):
            step()
        torch.cuda.synchronize()
        table = model.kernel_profile_read()
        model.kernel_profile(False)
        cand = [k for k in table if k in costs]
        dom = max(cand, key=lambda k: table[k][0]) if cand else None
        model.kernel_profile(True, only=dom)
    if ddp.is_distributed():
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if ddp.is_distributed():
        torch.distributed.barrier()
    el = time.perf_counter() - t0
    if ddp.is_distributed():
        t = torch.tensor([el], device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = t.item()
    prof = model.kernel_profile_read() if timing else {}  # the dominant kernel's launches in the timed region
    model.kernel_profile(False)
    final_loss = loss.item()

    if rank != 0:
        if ddp.is_distributed():
            torch.distributed.destroy_process_group()
        return

    ms_step = 1000.0 * el / args.steps
    nbuckets = len(bucketer.buckets(next(iter(model._plans.values())))) if bucketer is not None else 0
    backend = torch.distributed.get_backend() if ddp.is_distributed() else None
    if backend == "nccl":
        backend = "rccl"  # torch's "nccl" backend is RCCL on ROCm
    value = world * B * args.steps / el
    peak = BF16_PEAK_TFLOPS if bf16 else FP32_PEAK_TFLOPS
    roof = None
    kernels = {}
    if table:
        for lab, (tot, cnt) in sorted(table.items(), key=lambda kv: -kv[1][0]):
            kernels[lab] = {"avg_ms": round(tot / cnt, 4), "launches": cnt,
                            "share": round(tot / tsteps / ms_step, 4)}
    xfrac = (lambda lab: deep_executed_fraction(lab, F, T, bf16)) if deep else (lambda lab: executed_fraction(lab, T, F))
    if dom is not None and prof.get(dom):
        # the dominant kernel: the costed label with the largest total time in the table steps (every
        # kernel that matters has a cost model; the labels without one are tiny finalisers /
        # reductions), timed on its launch stream inside the timed region.  Its FLOPs are the ones it
        # EXECUTES (a Winograd F(2x2,3x3) kernel performs 16 multiplies per 2x2 outputs, 4/9 of the
        # direct conv's); the direct-conv-equivalent rate is reported beside it (alg_equiv_*).
        dom_any = max(table, key=lambda k: table[k][0])
        tot, cnt = prof[dom]
        avg_s = tot / cnt / 1000.0
        fl, by = costs[dom]
        xf = xfrac(dom)
        xfl = fl * xf
        if xfl / by > peak * 1e12 / (HBM_PEAK_GBS * 1e9):
            ach = xfl / avg_s / 1e12
            roof = {"kernel": dom, "bound": "mfma", "achieved": sig(ach), "peak": peak,
                    "unit": "TFLOP/s", "frac": sig(ach / peak), "flops_counted": "executed"}
        else:
            ach = by / avg_s / 1e9
            roof = {"kernel": dom, "bound": "hbm", "achieved": sig(ach), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": sig(ach / HBM_PEAK_GBS)}
        roof["traffic"] = load_pmc(args.model, args.precision if deep else "fp32", dom)
        roof["executed_flops_per_launch"] = int(xfl)
        roof["algorithmic_flops_per_launch"] = fl
        roof["algorithmic_bytes_per_launch"] = by
        if xf != 1.0:
            roof["alg_equiv_achieved"] = sig(fl / avg_s / 1e12)
            roof["alg_equiv_frac"] = sig(fl / avg_s / 1e12 / peak)
            roof["executed_per_algorithmic"] = round(xf, 6)
        roof["avg_launch_ms"] = round(avg_s * 1000.0, 4)
        roof["timed_launches"] = cnt
    if roof is not None:
        roof["largest_label_overall"] = dom_any
        for lab, rec in kernels.items():  # per-kernel achieved rates for every costed label
            if lab in costs:
                f_, b_ = costs[lab]
                t_ = rec["avg_ms"] / 1000.0
                if f_:
                    rec["exec_tflops"] = round(f_ * xfrac(lab) / t_ / 1e12, 2)
                    rec["exec_frac"] = round(f_ * xfrac(lab) / t_ / 1e12 / peak, 4)
                    rec["alg_tflops"] = round(f_ / t_ / 1e12, 2)
                rec["alg_gbps"] = round(b_ / t_ / 1e9, 1)
    # SURVEY 8(d)'s step byte model at the element size this path stores activations in (bf16 line:
    # e = 2, the survey's bf16 roof; fp32 lines: e = 4), and beside it the bytes the path actually
    # moves: the committed rocprofv3 PMC traffic per launch of every timed label x launches per step
    sf, sb = deep_step_cost(B, F, T, D, e=2 if bf16 else 4) if deep else step_cost(B, F, T, D)
    step_s = el / args.steps
    xsf = executed_step_flops(B, F, T, D, deep=deep, bf16=bf16)
    step_roof = {"flops_per_step": sf, "executed_flops_per_step": xsf, "bytes_per_step": sb,
                 "byte_model": "SURVEY 8(d), e=2 (bf16 activations)" if bf16 else "SURVEY 8(d), e=4 (fp32)",
                 # (schema 2: mfma_fraction is the algorithmic (direct-conv) FLOP rate, as in rounds 1-4; the
                 # round-5 lines wrote the executed rate under that key -- it is executed_mfma_fraction now)
                 "schema": 2,
                 "mfma_fraction": round(sf / step_s / (peak * 1e12), 4),
                 "executed_mfma_fraction": round(xsf / step_s / (peak * 1e12), 4),
                 "executed_counts": "Winograd kernels at 16 multiplies per 2x2 output tile (costs.wino_tile_fraction)",
                 "hbm_fraction": round(sb / step_s / (HBM_PEAK_GBS * 1e9), 4)}
    if table:
        mkey = (args.model, args.precision if deep else "fp32")
        moved, covered = 0.0, 0.0
        for lab, (tot, cnt) in table.items():
            t = load_pmc(*mkey, lab)
            if t:
                moved += t * cnt / tsteps
                covered += tot / tsteps
        if moved:
            step_roof["pmc_bytes_per_step"] = int(moved)
            step_roof["pmc_hbm_fraction"] = round(moved / step_s / (HBM_PEAK_GBS * 1e9), 4)
            step_roof["pmc_time_coverage"] = round(covered / ms_step, 4)

    peaks = None
    if rank == 0 and not args.no_peaks:
        try:
            peaks = measure_peaks(dev)
            if roof is not None:
                meas = peaks["fp32_gemm_TFLOPs"] if roof["bound"] == "mfma" and not bf16 else (
                    peaks["hbm_copy_GBps"] if roof["bound"] == "hbm" else None)
                if meas:
                    roof["frac_of_measured_peak"] = round(roof["achieved"] / meas, 4)
        except Exception as exc:  # pragma: no cover - reported, never fatal
            peaks = {"error": repr(exc)}

    cpu = None
    if world == 1 and not args.no_cpu_baseline and not deep:
        try:
            cpu = cpu_baseline(full=args.cpu_full, quick=args.cpu_quick)
        except Exception as exc:  # pragma: no cover - reported, never fatal for the GPU number
            cpu = {"error": repr(exc)}

    out = {
        "metric": METRIC if not deep else f"MFCC-samples/sec per train step (cnn_deep{', bf16 convs' if bf16 else ''}, batch {B})",
        "value": round(value, 1),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16 conv operands, fp32 accumulate/elsewhere" if bf16 else "fp32",
        "data": f"synthetic N(0,1) MFCC [B,1,40,T], random-init {args.model} (seed 42)",
        "config": {"workload": f"{args.model} contrastive train step: fwd + SupCon(T=0.15) + bwd + "
                               "grad all-reduce + Adam(lr 3e-4, wd 1e-4)",
                   "per_gpu_batch": B, "global_batch": B * world, "n_mfcc": F, "T": T,
                   "embedding_dim": D, "parallelism": f"dp{world}",
                   "allreduce": None if bucketer is None else f"{nbuckets} {backend} buckets behind the backward",
                   "allreduce_buckets": nbuckets,
                   "dist_backend": backend,
                   "dist_world_size": torch.distributed.get_world_size() if ddp.is_distributed() else 1,
                   "supcon": "global batch (embedding + coefficient all-gathers, anchor rows per rank)"
                             if args.global_supcon and world > 1 else "per rank (DDP-equivalent)"},
        "conv_algorithms": None if deep else {
            "conv_fwd / conv_dgrad L2-L6": "Winograd F(2x2,3x3) on fp32 MFMA (16 multiplies per 2x2 outputs: "
                                           "4/9 of the direct conv's; fp32 arithmetic, rounding differs from the direct "
                                           "conv by 2-6e-6 of max|y|)",
            "wgrad L2-L6": "Winograd F(2x2,3x3) weight gradient on fp32 MFMA (even W; 4/9 of the direct "
                           "multiplies), else the direct pixel-stream implicit GEMM"},
        "roofline": roof,
        "step_roofline": step_roof,
        "cpu_baseline": cpu,
        "measured_peaks": peaks,
        "kernels": kernels,
        "kernel_table": f"per-launch HIP-event times over {tsteps} untimed steps after the warm-up; the timed "
                        "region records the roofline kernel alone" if table else None,
        "final_loss": round(final_loss, 5),
    }
    print(json.dumps(out), flush=True)
    if ddp.is_distributed():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
