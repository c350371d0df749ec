"""Helpers to read the committed golden fixtures (tests/golden/*.npz, made by make_golden.py)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# biases that feed a train-mode BatchNorm have an analytically zero gradient; the reference's
# value is float noise, so they are compared against an absolute floor only
BN_FED_BIAS_FLOOR = 1e-4


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def section(d, prefix):
    p = prefix + "/"
    return {k[len(p):]: d[k] for k in d.files if k.startswith(p)}


def model_case(name):
    """Returns dict with x, labels, masks per step, state0, grads, emb/loss per step, meta."""
    d = load(name)
    base = {"cnn_small_T201": "cnn_small_T200", "cnn_deep_T201": "cnn_deep_T200"}.get(name)
    state0 = section(load(base) if base else d, "state0")
    B, T, temp, lr, wd = d["meta"]
    case = {"x": d["x"], "labels": d["labels"], "state0": state0, "grads": section(d, "grad"),
            "temperature": float(temp), "lr": float(lr), "weight_decay": float(wd),
            "steps": [], "state_final": section(d, "state_final"),
            "f64": {"emb": d["f64/emb"], "loss": float(d["f64/loss"][0]),
                    "grads": section(d, "f64/grad")}}
    s = 0
    while f"step{s}/loss" in d.files:
        st = section(d, f"step{s}")
        nm = sorted(k for k in st if k.startswith("mask"))
        case["steps"].append({"emb": st["emb"], "loss": float(st["loss"][0]),
                              "masks": [st[k] for k in nm]})
        s += 1
    return case


def bn_fed_bias(name, sd_keys):
    """True for a conv/linear bias whose output feeds a BatchNorm in train mode."""
    if not name.endswith(".bias"):
        return False
    stem = name[:-5]
    if stem.startswith("projection.0"):
        return True
    if stem.endswith("conv1") or stem.endswith("conv2") or stem.endswith("shortcut.0") \
            or stem == "init_conv.0":
        return True
    parts = stem.split(".")
    # conv_blocks.{i}.{0,3} in PhonemeNet
    return len(parts) == 3 and parts[0] == "conv_blocks" and parts[2] in ("0", "3")


def grad_errors(got, ref):
    """Per-tensor error: max|got-ref| / max|ref| (abs for BN-fed biases)."""
    out = {}
    for k, r in ref.items():
        g = np.asarray(got[k], dtype=np.float64).reshape(r.shape)
        if bn_fed_bias(k, ref):
            out[k] = ("abs", float(np.abs(g - r).max()))
        else:
            out[k] = ("rel", float(np.abs(g - r).max() / max(np.abs(r).max(), 1e-30)))
    return out
