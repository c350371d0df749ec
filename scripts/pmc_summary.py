#!/usr/bin/env python
"""Summarise rocprofv3 output of scripts/profile_gpu.sh into profiles/.

* kernel stats (trace pass) -> per-kernel average duration
* PMC passes -> HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
  (gfx950: FETCH_SIZE counts half the bytes of wide coalesced reads, MI355X_MICROARCH.md HBM)
Dispatches of one template instance are mapped to network layers by their order inside a step
(the plan's launch order is fixed: forward L1..L6, backward L6..L1).
"""
import csv
import json
import sys
from collections import defaultdict

# template instance -> layer labels in per-step dispatch order (cnn_small)
ORDER = {
    "conv3x3_kernel<1, 4, 1, 0>": ["conv_fwd_L2"],
    "conv3x3_kernel<2, 2, 2, 0>": ["conv_fwd_L3", "conv_fwd_L5"],
    "conv3x3_kernel<2, 2, 1, 0>": ["conv_fwd_L4", "conv_fwd_L6"],
    "conv3x3_kernel<2, 2, 3, 1>": ["conv_dgrad_L6", "conv_dgrad_L4"],
    "conv3x3_kernel<2, 2, 3, 2>": ["conv_dgrad_L5"],
    "conv3x3_kernel<1, 4, 3, 2>": ["conv_dgrad_L3"],
    "conv3x3_kernel<1, 4, 3, 1>": ["conv_dgrad_L2"],
    "wgrad3x3_kernel<32, 1, 1>": ["wgrad_L6", "wgrad_L4"],
    "wgrad3x3_kernel<32, 1, 2>": ["wgrad_L5"],
    "wgrad3x3_kernel<16, 2, 2>": ["wgrad_L3"],
    "wgrad3x3_kernel<16, 1, 1>": ["wgrad_L2"],
    "conv1_fwd_kernel": ["conv1_fwd_L1"],
    "wgrad1_kernel": ["wgrad_L1"],
}


def short(name):
    for k in ORDER:
        if k in name:
            return k
    return None


def counters(path, counter):
    per = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            k = short(r["Kernel_Name"])
            if k:
                per[k].append(float(r["Counter_Value"]))
    out = defaultdict(list)
    for k, vals in per.items():
        labs = ORDER[k]
        for i, v in enumerate(vals):
            out[labs[i % len(labs)]].append(v)
    return out


def main(prof_dir, out_json):
    fetch = counters(f"{prof_dir}/pmc_fetch/run_counter_collection.csv", "FETCH_SIZE")
    write = counters(f"{prof_dir}/pmc_write/run_counter_collection.csv", "WRITE_SIZE")
    res = {}
    for lab in sorted(set(fetch) | set(write)):
        f = sorted(fetch.get(lab, [0.0]))[len(fetch.get(lab, [0.0])) // 2]
        w = sorted(write.get(lab, [0.0]))[len(write.get(lab, [0.0])) // 2]
        res[lab] = {"fetch_size_kb": f, "write_size_kb": w,
                    "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024),
                    "note": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE half-count correction)"}
    with open(out_json, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
