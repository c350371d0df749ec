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

FP32_PEAK_TFLOPS = 157.3     # MI355X vector == matrix fp32 (MI355X_MICROARCH.md)
BF16_PEAK_TFLOPS = 2500.0    # dense bf16 MFMA (MI355X_MICROARCH.md: ~2.5 PF dense, no sparsity)
HBM_PEAK_GBS = 8000.0        # HBM3E spec
METRIC = "MFCC-samples/sec per train step (cnn_small, batch 4096) at 1/2/4/8 MI355X"
DEEP_DIMS = [64, 128, 256, 512]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ----------------------------------------------------------------------------- algorithmic cost
def small_layers(B, F, T):
    """(label suffix, cin, cout, H, W, src bytes/sample, pooled) for the six convs of cnn_small."""
    H1, W1 = F, T
    H3, W3 = H1 // 2, W1 // 2
    H5, W5 = H3 // 2, W3 // 2
    return [(1, 1, 32, H1, W1), (2, 32, 32, H1, W1), (3, 32, 64, H3, W3), (4, 64, 64, H3, W3),
            (5, 64, 128, H5, W5), (6, 128, 128, H5, W5)]


def kernel_costs(B, F, T, D=128):
    """Algorithmic FLOPs and HBM bytes of ONE launch of each profiled kernel label.
    FLOPs: 2*MACs of the dense contraction.  Bytes: each input tensor read once, each output
    written once, fp32 (halo / prologue re-reads are not algorithmic)."""
    L = {l: (ci, co, h, w) for l, ci, co, h, w in small_layers(B, F, T)}
    src_res = {1: (F, T), 2: (F, T), 3: (F, T), 4: (F // 2, T // 2), 5: (F // 2, T // 2), 6: (F // 4, T // 4)}
    out = {}
    for l, (ci, co, h, w) in L.items():
        macs = B * h * w * co * ci * 9
        sh, sw = src_res[l]
        y_out = 4 * B * co * h * w
        x_in = 4 * B * ci * sh * sw
        if l == 1:
            out["conv1_fwd_L1"] = (2 * macs, 4 * B * F * T + y_out)
            out["wgrad_L1"] = (2 * macs, 2 * y_out + 4 * B * F * T)
            continue
        out[f"conv_fwd_L{l}"] = (2 * macs, x_in + y_out)
        # dgrad: reads dz_l and y_l, reads y_{l-1} (epilogue), writes dz_{l-1}
        out[f"conv_dgrad_L{l}"] = (2 * macs, 2 * y_out + 2 * x_in)
        # wgrad: reads dz_l, y_l and the forward input source
        out[f"wgrad_L{l}"] = (2 * macs, 2 * y_out + x_in)
    # elementwise / head passes (bytes: each tensor read once, each output written once)
    H1, W1, H3, W3, H5, W5 = F, T, F // 2, T // 2, F // 4, T // 4
    out["bn_relu_pool_L3"] = (0, 4 * B * 32 * (H1 * W1 + H3 * W3))
    out["bn_relu_pool_L5"] = (0, 4 * B * 64 * (H3 * W3 + H5 * W5))
    out["head_pool_fwd"] = (4 * B * 128 * H5 * W5, 4 * B * (128 * H5 * W5 + 128 + H5 * W5))
    out["head_pool_bwd"] = (6 * B * 128 * H5 * W5, 4 * B * (2 * 128 * H5 * W5 + 128 + H5 * W5))
    out["proj_fwd"] = (2 * B * 128 * D, 4 * B * (128 + 2 * D))
    out["proj_bwd"] = (4 * B * 128 * D, 4 * B * (2 * 128 + 3 * D))
    return out


def executed_fraction(label, T):
    """Multiplies executed per algorithmic (direct-conv) multiply for cnn_small's kernels: the 3x3
    forward / data-gradient convs run Winograd F(2x2,3x3) at W >= 31 (conv_wino.hip), the 3x3
    weight gradients at even W (wgrad_wino.hip): 16 multiplies per 2x2 outputs instead of 36."""
    widths = {2: T, 3: T // 2, 4: T // 2, 5: T // 4, 6: T // 4}
    for pre in ("conv_fwd_L", "conv_dgrad_L"):
        if label.startswith(pre):
            return 4 / 9 if widths.get(int(label[len(pre):]), 0) >= 31 else 1.0
    if label.startswith("wgrad_L") and label[7:].isdigit() and int(label[7:]) >= 2:
        return 4 / 9 if widths[int(label[7:])] % 2 == 0 else 1.0
    return 1.0


def deep_convs(F, T, h=DEEP_DIMS):
    """(fwd label, wgrad label, dgrad label or None, cin, cout, k, stride, IH, IW, OH, OW) of every
    conv of cnn_deep, labelled as deep.hip profiles them."""
    out = [("conv_fwd_L0", "wgrad_L0", None, 1, h[0], 7, 1, F, T, F, T)]
    H, W, cin = (F - 1) // 2 + 1, (T - 1) // 2 + 1, h[0]
    for i, co in enumerate(h):
        s = 1 if i == 0 else 2
        Ho, Wo = (H - 1) // s + 1, (W - 1) // s + 1
        L = 2 * i + 1
        out.append((f"conv_fwd_L{L}", f"wgrad_L{L}", f"conv_dgrad_L{L}", cin, co, 3, s, H, W, Ho, Wo))
        out.append((f"conv_fwd_L{L + 1}", f"wgrad_L{L + 1}", f"conv_dgrad_L{L + 1}", co, co, 3, 1, Ho, Wo, Ho, Wo))
        if s != 1 or cin != co:
            out.append((f"shortcut_fwd_L{i}", f"wgrad_L{100 + i}", f"conv_dgrad_L{100 + i}", cin, co, 1, s, H, W,
                        Ho, Wo))
        H, W, cin = Ho, Wo, co
    return out


def deep_kernel_costs(B, F, T, bf16=False, D=128):
    """Algorithmic FLOPs and bytes of one launch of every profiled cnn_deep label (convs: both
    operands read once, the output written once, float32; elementwise passes: each tensor read
    once, each output written once, float32 activations, bf16 channel-last images 2 B/element)."""
    out = {}
    for fl, wl, dl, ci, co, k, s, IH, IW, OH, OW in deep_convs(F, T):
        macs = B * OH * OW * co * ci * k * k
        x_b, y_b = 4 * B * ci * IH * IW, 4 * B * co * OH * OW
        out[fl] = (2 * macs, x_b + y_b)
        out[wl] = (2 * macs, x_b + y_b)
        if dl:
            out[dl] = (2 * macs, x_b + y_b)
    img = 2 if bf16 else 4
    H0, W0 = F, T
    H1, W1 = (H0 - 1) // 2 + 1, (W0 - 1) // 2 + 1
    C0 = DEEP_DIMS[0]
    out["maxpool_fwd"] = (0, B * C0 * (4 * H0 * W0 + 5 * H1 * W1))            # y0 -> a0 + first-max tap
    out["maxpool_bwd"] = (0, B * C0 * (4 * H0 * W0 * 2 + 9 * H1 * W1))        # tap, d a0 + shortcut grad, y0 -> dz0
    if bf16 and C0 == 64 and W0 <= 256:
        # fused stem (conv.hip stem_pool_kernel / stem_wgrad_rc_kernel): y0 is recomputed, never stored;
        # the stem GEMM's FLOPs count once per recomputation
        stem = 2 * B * H0 * W0 * C0 * 49
        xb = 4 * B * H0 * W0
        out["conv_fwd_L0"] = (stem, xb)                                        # BN0 statistics only
        # pooled NHWC y0 at the tap (4 B) + tap (1 B) + block 0's NHWC image; no a0 plane
        out["maxpool_fwd"] = (stem, xb + B * C0 * (5 * H1 * W1 + img * (H1 + 2) * (W1 + 2)))
        # d a0 + block 0's shortcut gradient + tap + y0 at the tap -> dz0 in bf16
        out["maxpool_bwd"] = (0, B * C0 * (13 * H1 * W1 + 2 * H0 * W0))
        out["wgrad_L0"] = (2 * stem, xb + 2 * B * C0 * H0 * W0)                # bf16 dz0 + x (recompute + gradient)
    out["bwd_prep_L0"] = (0, B * C0 * 4 * H0 * W0 * 3)
    H, W, cin = H1, W1, C0
    for i, co in enumerate(DEEP_DIMS):
        st = 1 if i == 0 else 2
        Ho, Wo = (H - 1) // st + 1, (W - 1) // st + 1
        L, Pi, Po = 2 * i + 1, H * W, Ho * Wo
        sc = st != 1 or cin != co
        a_in, y = 4 * B * cin * Pi, 4 * B * co * Po
        out[f"to_nhwc_L{L}"] = (0, a_in + img * B * cin * (H + 2) * (W + 2))
        out[f"bn_act_L{L}"] = (0, y + img * B * co * Po)                         # y1 -> d1
        # bf16: outputs of even-width blocks 0-1 leave a byte ReLU mask instead of the float32 plane
        m8 = bf16 and i < 2 and Wo % 2 == 0
        out[f"bn_act_L{L + 1}"] = (0, 2 * y + (y // 4 if m8 else y) + img * B * co * Po)  # y2 + residual -> out / mask (+ image)
        out[f"chan_stats_L{L}"] = (0, y)
        out[f"chan_stats_L{L + 1}"] = (0, y)
        out[f"chan_stats_L{100 + i}"] = (0, y)
        out[f"bwd_prep_L{L + 1}"] = (0, y * (4 if sc else 3) + y - (3 * y // 4 if m8 else 0))  # d, mask, y2 (, ysc) -> g
        out[f"bwd_prep_L{L}"] = (0, (2 if bf16 else 3) * y)                      # d, y1 (-> d; bf16: sums only)
        out[f"dy_nhwc_L{L + 1}"] = (0, 2 * y + img * B * co * Po)
        out[f"dy_nhwc_L{L}"] = (0, 2 * y + img * B * co * Po)
        out[f"bn_bwd_apply_L{L + 1}"] = (0, 3 * y)
        out[f"bn_bwd_apply_L{L}"] = (0, 3 * y)
        out[f"dgrad_interleave_L{L}"] = (0, 2 * a_in)
        H, W, cin = Ho, Wo, co
    C4, P4 = DEEP_DIMS[-1], H * W
    out["head_pool_fwd"] = (4 * B * C4 * P4, 4 * B * (C4 * P4 + C4 + P4))
    out["head_pool_bwd"] = (6 * B * C4 * P4, 4 * B * (2 * C4 * P4 + C4 + P4))
    out["proj_fwd"] = (2 * B * C4 * D, 4 * B * (C4 + 2 * D))
    out["proj_bwd"] = (4 * B * C4 * D, 4 * B * (2 * C4 + 3 * D))
    return out


def deep_step_cost(B, F, T, D=128, e=4):
    """SURVEY 8(d)'s cnn_deep model: input read twice, every conv output written / read / re-read /
    gradient written / read (5 passes), the same for the init max-pool output and every block
    output; + 40 B per parameter and 12 B*D for SupCon (122.37 GB / step at B = 4096, T = 200)."""
    flops, act = 0, e * 2 * B * F * T
    for fl, wl, dl, ci, co, k, s, IH, IW, OH, OW in deep_convs(F, T):
        macs = B * OH * OW * co * ci * k * k
        flops += 2 * macs * (3 if dl else 2)
        act += e * 5 * B * co * OH * OW
    H, W = (F - 1) // 2 + 1, (T - 1) // 2 + 1
    act += e * 5 * B * DEEP_DIMS[0] * H * W  # init max-pool output
    for i, co in enumerate(DEEP_DIMS):
        s = 1 if i == 0 else 2
        H, W = (H - 1) // s + 1, (W - 1) // s + 1
        act += e * 5 * B * co * H * W        # block output
    flops += 4 * B * B * D + 3 * 2 * B * DEEP_DIMS[-1] * D
    return flops, act + 40 * 4968833 + 12 * B * D


def step_cost(B, F, T, D=128):
    """Algorithmic FLOPs and bytes of one whole train step."""
    flops = 0
    act_bytes = 4 * 2 * B * F * T  # input read twice
    for l, ci, co, h, w in small_layers(B, F, T):
        macs = B * h * w * co * ci * 9
        flops += 2 * macs * (2 if l == 1 else 3)
        act_bytes += 4 * 5 * B * co * h * w
    flops += 4 * B * B * D + 3 * 2 * B * 128 * D
    params = 304225
    return flops, act_bytes + 40 * params + 12 * B * D


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
    tr.step(x, labels, masks)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        tr.step(x, labels, masks)
        n += 1
        el = time.perf_counter() - t0
        if (el >= min_s and n >= min_steps) or n >= max_steps:
            break
    return {"B": B, "threads": threads, "steps": n, "seconds": round(el, 2), "samples_per_s": round(B * n / el, 2)}


def cpu_baseline(full=False, T=200):
    """The reference step on the host cores (the reference itself cannot travel to the GPU box):
    the float32 torch-CPU restatement (oracle/torch_port.py, pinned to the reference's fixtures),
    at the reference's real train batch B = 24 (6 classes x 2 clips x 2 views) with cores - 2
    threads (src/utils/device.py:58-61) and with all cores; `full` adds the BASELINE's B = 4096
    (1 warm-up + 2 timed steps per thread count: several minutes)."""
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 2)
    allc = max(1, min(share, os.cpu_count() or share))
    rule = max(1, allc - 2)
    legs = [_cpu_leg(24, T, rule, 6.0, 3), _cpu_leg(24, T, allc, 6.0, 3)]
    if full:
        legs += [_cpu_leg(4096, T, rule, 0.0, 2, 2), _cpu_leg(4096, T, allc, 0.0, 2, 2)]
    main = legs[0]
    return {"value": main["samples_per_s"], "unit": "samples/s", "cores": main["threads"], "kind": "port",
            "cpu_model": cpu_model_name(), "host_threads_available": allc,
            "sample": f"cnn_small train step (fwd+SupCon+bwd+Adam) at the reference's real batch B=24, T={T}, "
                      f"{main['steps']} steps in {main['seconds']}s on cores-2 = {main['threads']} threads "
                      "(reference rule, src/utils/device.py:58-61); float32 torch-CPU restatement "
                      "oracle/torch_port.py", "legs": legs}


def measure_peaks(dev):
    """Achievable peaks on this box (report against vendor and measured): HBM by a
    2 GiB device-to-device copy, fp32 matrix rate by an 8192^3 torch.mm (rocBLAS / hipBLASLt
    fp32 GEMM on the MFMA).  Timed with HIP events after a warm-up; ~1 s in total."""
    n = 1 << 29  # floats: 2 GiB per buffer
    a = torch.empty(n, device=dev)
    b = torch.empty(n, device=dev)
    b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    hbm = 5 * 2 * 4 * n / (e0.elapsed_time(e1) / 1000.0) / 1e9
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
    return {"hbm_copy_GBps": round(hbm, 1), "fp32_gemm_TFLOPs": round(gemm, 1),
            "note": "measured on this GPU: 2 GiB D2D copy (read + write bytes); torch.mm fp32 8192^3"}


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
    ap.add_argument("--cpu-full", action="store_true", help="also time the CPU baseline at B=4096 (minutes)")
    ap.add_argument("--bucket-mb", type=float, default=None,
                    help="N > 1: gradient all-reduce bucket size (default 0.5 MB cnn_small, 4 MB cnn_deep)")
    ap.add_argument("--global-supcon", action="store_true",
                    help="N > 1: SupCon over the global batch (embedding all-gather, sharded anchor rows)")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--no-peaks", action="store_true", help="skip the measured-peak probes")
    args = ap.parse_args()

    from phoneme_contrast_amd import distributed as ddp
    from phoneme_contrast_amd.losses import GlobalSupervisedContrastiveLoss, SupervisedContrastiveLoss
    from phoneme_contrast_amd.models import model_registry
    from phoneme_contrast_amd.optim import FusedAdam

    rank, world, local = ddp.init_from_env()
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}")
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

    timing = not args.no_kernel_timing
    if timing:
        model.kernel_profile(True)
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
    prof = model.kernel_profile_read() if timing else {}
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
    bf16 = deep and args.precision == "bf16"
    costs = deep_kernel_costs(B, F, T, bf16, D) if deep else kernel_costs(B, F, T, D)
    peak = BF16_PEAK_TFLOPS if bf16 else FP32_PEAK_TFLOPS
    roof = None
    kernels = {}
    if prof:
        for lab, (tot, cnt) in sorted(prof.items(), key=lambda kv: -kv[1][0]):
            kernels[lab] = {"avg_ms": round(tot / cnt, 4), "launches": cnt,
                            "share": round(tot / (1000.0 * el), 4)}
        # the dominant kernel: the label with the largest total time (every kernel that matters has
        # a cost model; the bookkeeping labels without one are the tiny finalisers / reductions)
        dom_any = max(prof, key=lambda k: prof[k][0])
        dom = max((k for k in prof if k in costs), key=lambda k: prof[k][0])
        tot, cnt = prof[dom]
        avg_s = tot / cnt / 1000.0
        fl, by = costs[dom]
        ai = fl / by
        if ai > peak * 1e12 / (HBM_PEAK_GBS * 1e9):
            ach = fl / avg_s / 1e12
            roof = {"kernel": dom, "bound": "mfma", "achieved": round(ach, 2), "peak": peak,
                    "unit": "TFLOP/s", "frac": round(ach / peak, 4)}
        else:
            ach = by / avg_s / 1e9
            roof = {"kernel": dom, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4)}
        roof["traffic"] = load_pmc(args.model, args.precision if deep else "fp32", dom)
        roof["algorithmic_flops_per_launch"] = fl
        roof["algorithmic_bytes_per_launch"] = by
        roof["avg_launch_ms"] = round(avg_s * 1000.0, 4)
    if roof is not None:
        roof["largest_label_overall"] = dom_any
        if not deep and roof["bound"] == "mfma":
            # cnn_small's 3x3 convs run Winograd F(2x2,3x3): 4/9 of the direct multiplies are executed
            xf = executed_fraction(dom, T)
            roof["executed_flops_per_launch"] = int(fl * xf)
            roof["executed_frac"] = round(roof["frac"] * xf, 4)
        for lab, rec in kernels.items():  # per-kernel achieved rates for every costed label
            if lab in costs:
                f_, b_ = costs[lab]
                t_ = rec["avg_ms"] / 1000.0
                rec["alg_tflops"] = round(f_ / t_ / 1e12, 2) if f_ else None
                rec["alg_gbps"] = round(b_ / t_ / 1e9, 1)
    sf, sb = deep_step_cost(B, F, T, D) if deep else step_cost(B, F, T, D)
    step_roof = {"flops_per_step": sf, "bytes_per_step": sb,
                 "mfma_fraction": round(sf / (el / args.steps) / (peak * 1e12), 4),
                 "hbm_fraction": round(sb / (el / args.steps) / (HBM_PEAK_GBS * 1e9), 4)}

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
            cpu = cpu_baseline(full=args.cpu_full)
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
        "final_loss": round(final_loss, 5),
    }
    print(json.dumps(out), flush=True)
    if ddp.is_distributed():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
