#!/usr/bin/env python
"""Summarise rocprofv3 output of scripts/profile_gpu.sh into profiles/.

* PMC passes -> HBM bytes per launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
  (gfx950: FETCH_SIZE counts half the bytes of wide coalesced reads, MI355X_MICROARCH.md HBM)
* kernel trace -> per-layer average duration (to check against bench.py's live HIP-event timing)

Dispatches of a kernel family are mapped to network layers by their order inside a step (the
cnn_small plan's launch order is fixed: forward L1..L6, backward L6..L1), ordered by dispatch id.
"""
import csv
import json
import sys
from collections import defaultdict

FWD = [f"conv_fwd_L{l}" for l in range(2, 7)]
DGRAD = [f"conv_dgrad_L{l}" for l in range(6, 1, -1)]
# kernel family (name up to '<' / '(') -> layer labels in per-step dispatch order
ORDER = {
    # Winograd conv (every cnn_small layer at W >= 31); layer 2's data gradient runs inside the fused
    # layer-2 backward (wgbd_wino_kernel, round 4) at T = 200
    "conv_wino_kernel": FWD + DGRAD[:-1],
    "conv3x3_dma_kernel": FWD + DGRAD,
    "wgrad_s_kernel": [f"wgrad_L{l}" for l in range(6, 1, -1)],
    "wgrad_wino_kernel": [f"wgrad_L{l}" for l in range(6, 2, -1)],  # Winograd weight gradient (W even)
    "wgbd_wino_kernel": ["wgbd_L2"],
    "wgrad_wino_reduce_kernel": [f"wgrad_reduce_L{l}" for l in range(6, 1, -1)],
    "bn_relu_pool_kernel": ["bn_relu_pool_L3", "bn_relu_pool_L5"],
    "conv1_fwd_kernel": ["conv1_fwd_L1"],
    "wgrad1_kernel": ["wgrad_L1"],
    "supcon_rows_partial": ["supcon_rows"],
    "supcon_grad_partial": ["supcon_grad"],
    "adam_kernel": ["adam"],
}


def order_for(per):
    """Layer labels per family (one weight-gradient kernel, wgrad_s, serves L6..L2)."""
    return dict(ORDER)


def family(name):
    name = name.replace("(anonymous namespace)", "")
    base = name.split("(")[0].split("<")[0].split("::")[-1].strip()
    return base if base in ORDER else None


def _rows(path):
    with open(path) as f:
        rows = list(csv.DictReader(f))
    key = "Dispatch_Id" if rows and "Dispatch_Id" in rows[0] else None
    if key:
        rows.sort(key=lambda r: int(r[key]))
    return rows


def counters(path, counter):
    per = defaultdict(list)
    for r in _rows(path):
        if r.get("Counter_Name") != counter:
            continue
        k = family(r["Kernel_Name"])
        if k:
            per[k].append(float(r["Counter_Value"]))
    out = defaultdict(list)
    order = order_for(per)
    for k, vals in per.items():
        labs = order[k]
        for i, v in enumerate(vals):
            out[labs[i % len(labs)]].append(v)
    return out


def durations(path):
    per = defaultdict(list)
    for r in _rows(path):
        k = family(r["Kernel_Name"])
        if k:
            per[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = defaultdict(list)
    order = order_for(per)
    for k, vals in per.items():
        labs = order[k]
        for i, v in enumerate(vals):
            out[labs[i % len(labs)]].append(v)
    return {k: {"avg_ms": round(sum(v) / len(v), 4), "launches": len(v)} for k, v in out.items()}


def main(prof_dir, out_json, out_dur=None, key="cnn_small/fp32"):
    """Writes {key: {label: traffic}} into out_json (merged with the other workloads already
    there: bench.py looks traffic up by (model, precision, label))."""
    fetch = counters(f"{prof_dir}/pmc_fetch/run_counter_collection.csv", "FETCH_SIZE")
    write = counters(f"{prof_dir}/pmc_write/run_counter_collection.csv", "WRITE_SIZE")
    res = {}
    for lab in sorted(set(fetch) | set(write)):
        f = sorted(fetch.get(lab, [0.0]))[len(fetch.get(lab, [0.0])) // 2]
        w = sorted(write.get(lab, [0.0]))[len(write.get(lab, [0.0])) // 2]
        res[lab] = {"fetch_size_kb": f, "write_size_kb": w,
                    "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024),
                    "note": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE half-count correction)"}
    try:
        with open(out_json) as fi:
            allres = json.load(fi)
    except (OSError, ValueError):
        allres = {}
    allres[key] = res
    with open(out_json, "w") as fo:
        json.dump(allres, fo, indent=1)
    print(json.dumps(res, indent=1))
    if out_dur:
        d = durations(f"{prof_dir}/trace/run_kernel_trace.csv")
        with open(out_dur, "w") as fo:
            json.dump(d, fo, indent=1)
        print(json.dumps(d, indent=1))


def labelled(rename_trace, csv_path, counter):
    """Per-label values of `counter` from a --pmc pass, keyed by the labels of a kernel trace of the
    same command run with PCX_ROCTX=1 under `--marker-trace --kernel-rename` (the plan's labels as
    ROCTx ranges): both runs dispatch the same sequence, so dispatch k of one is dispatch k of the
    other.  Unlabelled dispatches keep their kernel family name; a name mismatch there aborts."""
    names = [r["Kernel_Name"] for r in _rows(rename_trace)]
    disp = defaultdict(dict)
    for r in _rows(csv_path):
        disp[int(r["Dispatch_Id"])].setdefault("name", r["Kernel_Name"])
        if r.get("Counter_Name") == counter:
            disp[int(r["Dispatch_Id"])]["v"] = disp[int(r["Dispatch_Id"])].get("v", 0.0) + float(r["Counter_Value"])
    ids = sorted(disp)
    if len(ids) != len(names):
        raise SystemExit(f"dispatch counts differ: trace {len(names)} vs pmc {len(ids)}")
    out = defaultdict(list)
    prev = None
    for lab, i in zip(names, ids):
        pname = disp[i]["name"]
        base = lambda n: n.replace("(anonymous namespace)", "").split("(")[0].split("<")[0].split("::")[-1].strip()
        renamed = not ("(" in lab or "<" in lab or "::" in lab)
        if not renamed:  # not renamed: must be the same kernel
            if base(lab) != base(pname):
                raise SystemExit(f"dispatch {i}: trace {base(lab)} vs pmc {base(pname)}")
            lab = base(lab)
        if "v" in disp[i]:
            if lab == prev and renamed:  # consecutive dispatches of one labelled scope: one launch
                out[lab][-1] += disp[i]["v"]
            else:
                out[lab].append(disp[i]["v"])
        prev = lab
    return out


def main_labelled(rename_trace, prof_dir, out_json, key):
    fetch = labelled(rename_trace, f"{prof_dir}/pmc_fetch/run_counter_collection.csv", "FETCH_SIZE")
    write = labelled(rename_trace, f"{prof_dir}/pmc_write/run_counter_collection.csv", "WRITE_SIZE")
    res = {}
    for lab in sorted(set(fetch) | set(write)):
        fv, wv = sorted(fetch.get(lab, [0.0])), sorted(write.get(lab, [0.0]))
        f, w = fv[len(fv) // 2], wv[len(wv) // 2]
        res[lab] = {"fetch_size_kb": f, "write_size_kb": w, "launches_seen": len(fv),
                    "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024),
                    "note": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE half-count correction); "
                            "median over the launches of the label (summed over its dispatches)"}
    try:
        with open(out_json) as fi:
            allres = json.load(fi)
    except (OSError, ValueError):
        allres = {}
    allres[key] = res
    with open(out_json, "w") as fo:
        json.dump(allres, fo, indent=1)
    print(json.dumps(res, indent=1))


def stalls(csv_path, out_json):
    """Median of every counter of one --pmc pass, per layer label (analysis aid)."""
    names = sorted({r["Counter_Name"] for r in _rows(csv_path)})
    res = defaultdict(dict)
    for c in names:
        for lab, vals in counters(csv_path, c).items():
            res[lab][c] = sorted(vals)[len(vals) // 2]
    for lab, d in res.items():
        if d.get("SQ_WAVE_CYCLES"):
            for c in list(d):
                if c.startswith("SQ_WAIT") or c.startswith("SQ_ACTIVE"):
                    d[c + "/WAVE_CYCLES"] = round(d[c] / d["SQ_WAVE_CYCLES"], 4)
        if d.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in d:
            # MFMA busy per SIMD: 1024 SIMDs x (GRBM_GUI_ACTIVE / 8 XCDs)
            d["mfma_busy_frac"] = round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / (128.0 * d["GRBM_GUI_ACTIVE"]), 4)
    with open(out_json, "w") as fo:
        json.dump(res, fo, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


def label_stalls(rename_trace, csv_path, out_json, key):
    """Per plan label: median per launch of every counter of one --pmc pass (dispatches mapped to the
    labels of a rename trace, as `labelled`), plus the wait / active fractions of wave cycles."""
    names = sorted({r["Counter_Name"] for r in _rows(csv_path)})
    res = defaultdict(dict)
    for c in names:
        for lab, vals in labelled(rename_trace, csv_path, c).items():
            res[lab][c] = sorted(vals)[len(vals) // 2]
    durs = defaultdict(list)  # per-label launch durations (ms) from the rename trace's timestamps
    prev = None
    for r in _rows(rename_trace):
        lab = r["Kernel_Name"]
        dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        if lab == prev and not ("(" in lab or "<" in lab or "::" in lab):
            durs[lab][-1] += dt
        else:
            durs[lab].append(dt)
        prev = lab
    for lab, d in res.items():
        if d.get("SQ_WAVE_CYCLES"):
            for c in list(d):
                if c.startswith("SQ_WAIT") or c.startswith("SQ_ACTIVE"):
                    d[c + "/WAVE_CYCLES"] = round(d[c] / d["SQ_WAVE_CYCLES"], 4)
        if d.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in d:
            # MFMA busy per SIMD: 1024 SIMDs x (GRBM_GUI_ACTIVE / 8 XCDs); a value at 2^31 / 2^32 is a
            # saturated counter (round 3 at B = 4096), not a measurement
            v = d["SQ_VALU_MFMA_BUSY_CYCLES"]
            d["mfma_busy_saturated"] = v >= 2.0 ** 31 - 1
            d["mfma_busy_frac"] = round(v / (128.0 * d["GRBM_GUI_ACTIVE"]), 4)
        if durs.get(lab):
            dv = sorted(durs[lab])
            d["trace_ms"] = round(dv[len(dv) // 2], 4)
            if d.get("GRBM_GUI_ACTIVE"):
                d["clock_ghz"] = round(d["GRBM_GUI_ACTIVE"] / 8.0 / (d["trace_ms"] * 1e6), 3)
            if d.get("SQ_INSTS_VALU_MFMA_MOPS_F32"):
                # fp32 MFMA work the hardware counted (units of 512 FLOPs): the executed FLOPs of the launch,
                # independent of the cost model, and their rate against the 157.3 TFLOP/s fp32 peak
                fl = d["SQ_INSTS_VALU_MFMA_MOPS_F32"] * 512.0
                d["mops_f32_flops"] = fl
                d["mops_f32_frac"] = round(fl / (d["trace_ms"] * 1e-3) / 157.3e12, 4)
            if d.get("SQ_INSTS_VALU_MFMA_MOPS_BF16"):
                fl = d["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512.0
                d["mops_bf16_flops"] = fl
                d["mops_bf16_frac"] = round(fl / (d["trace_ms"] * 1e-3) / 2500e12, 4)
    try:
        with open(out_json) as fi:
            allres = json.load(fi)
    except (OSError, ValueError):
        allres = {}
    allres[key] = res
    with open(out_json, "w") as fo:
        json.dump(allres, fo, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    if sys.argv[1] == "--stalls":
        stalls(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "--label-stalls":
        label_stalls(*sys.argv[2:6])
    elif sys.argv[1] == "--labels":
        main_labelled(*sys.argv[2:6])
    else:
        main(*sys.argv[1:5])
