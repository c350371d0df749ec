#!/usr/bin/env python
"""Speed of the CPU baseline port against the reference itself (the port stands in for
the reference on the GPU box only if it times within +-10 % of the reference's own CPU step here).

Runs in THIS container only (the reference never travels): imports the reference's PhonemeNet and
SupervisedContrastiveLoss from /root/reference (read-only; no bytecode is written there) and times
its raw train step -- forward, SupCon, zero_grad, backward, Adam.step, loss.item(), i.e.
/root/reference/src/training/trainer.py:136-160 without the data loader -- against
oracle/torch_port.CpuTrainer.step on identical weights and inputs, with the same thread counts,
legs interleaved (ref, port, ref, port) to cancel drift.  Writes profiles/cpu_port_vs_reference.json.

    python scripts/cpu_port_vs_reference.py [--seconds 4] [--out profiles/cpu_port_vs_reference.json]
"""
import argparse
import json
import os
import platform
import sys
import time

sys.dont_write_bytecode = True
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

import torch  # noqa: E402


def timed(step, seconds, min_steps=3):
    step()  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        step()
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds and n >= min_steps:
            return n, el


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--batches", default="24,256")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "cpu_port_vs_reference.json"))
    args = ap.parse_args()
    sys.path.insert(0, ROOT)
    sys.path.insert(0, REF)
    from src.models.phoneme_cnn import PhonemeNet as RefNet  # the reference (read-only import)
    from src.training.losses import SupervisedContrastiveLoss as RefLoss

    from oracle import torch_port as tp

    cores = os.cpu_count() or 2
    legs = []
    for B in [int(b) for b in args.batches.split(",")]:
        for threads in sorted({max(1, cores - 2), cores}):
            torch.set_num_threads(threads)
            torch.manual_seed(42)
            ref = RefNet({"in_channels": 1, "embedding_dim": 128, "use_attention": True, "dropout_rate": 0.1}).train()
            sd = {k: v.detach().clone() for k, v in ref.state_dict().items()}
            opt = torch.optim.Adam(ref.parameters(), lr=3e-4, weight_decay=1e-4)
            loss_fn = RefLoss(temperature=0.15)
            port = tp.CpuTrainer(sd, temperature=0.15)
            g = torch.Generator().manual_seed(1234)
            x = torch.randn(B, 1, 40, 200, generator=g)
            labels = torch.arange(B // 4).repeat_interleave(4)
            masks = [(torch.rand(B, c, generator=g) >= 0.1).float() / 0.9 for c in (32, 64, 128)]

            def ref_step():
                e = ref(x)
                loss = loss_fn(e, labels)
                opt.zero_grad()
                loss.backward()
                opt.step()
                return loss.item()

            def port_step():
                return port.step(x, labels, masks).item()

            res = {"ref": [], "port": []}
            for _ in range(2):
                for name, fn in (("ref", ref_step), ("port", port_step)):
                    n, el = timed(fn, args.seconds / 2)
                    res[name].append(B * n / el)
            r = sum(res["ref"]) / len(res["ref"])
            p = sum(res["port"]) / len(res["port"])
            leg = {"B": B, "threads": threads, "reference_samples_per_s": round(r, 2),
                   "port_samples_per_s": round(p, 2), "port_over_reference": round(p / r, 4),
                   "within_10pct": abs(p / r - 1.0) <= 0.10}
            print(json.dumps(leg), flush=True)
            legs.append(leg)
    out = {"what": "raw train step (fwd + SupCon + zero_grad + bwd + Adam + loss.item) of the reference "
                   "(/root/reference/src/models/phoneme_cnn.py + src/training/losses.py, imported read-only) "
                   "vs oracle/torch_port.CpuTrainer, same weights / inputs / threads, legs interleaved",
           "cpu": platform.processor() or "unknown", "host_threads": cores, "torch": torch.__version__,
           "legs": legs, "all_within_10pct": all(leg["within_10pct"] for leg in legs)}
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    out["cpu"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({"all_within_10pct": out["all_within_10pct"]}))


if __name__ == "__main__":
    main()
