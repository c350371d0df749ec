"""float64 numpy restatement of PhonemeNet / PhonemeNetDeep train step (test oracle).

State is a reference-format state_dict (name -> ndarray), so fixtures generated from the
reference (`tests/golden/make_golden.py`) load directly.  Forward, SupCon, backward and Adam
are all explicit; see np_ops.py for the per-op citations.

  cnn_small: src/models/phoneme_cnn.py:10-126  (3 conv blocks, SpatialAttention, projection)
  cnn_deep : src/models/phoneme_cnn.py:146-304 (init conv7x7 + maxpool(3,2,1), ResidualBlocks)
"""
import numpy as np

from . import np_ops as op


def _f64(sd):
    return {k: np.asarray(v, dtype=np.float64) if np.asarray(v).dtype.kind == "f" else np.asarray(v)
            for k, v in sd.items()}


def param_names(sd):
    """Parameter (trainable) names in state_dict order, i.e. model.named_parameters() order."""
    return [k for k in sd if not (k.endswith("running_mean") or k.endswith("running_var")
                                  or k.endswith("num_batches_tracked"))]


def is_deep(sd):
    return "init_conv.0.weight" in sd


# ----------------------------------------------------------------------------- shared pieces
class _Tape:
    def __init__(self):
        self.ops = []
        self.stats = {}

    def push(self, *rec):
        self.ops.append(rec)


def _conv(t, sd, name, x, stride, pad):
    y = op.conv2d_fwd(x, sd[name + ".weight"], sd[name + ".bias"], stride, pad)
    t.push("conv", name, x, stride, pad)
    return y


def _bn(t, sd, name, x, train, axes):
    if not train:
        return op.bn_eval(x, sd[name + ".weight"], sd[name + ".bias"],
                          sd[name + ".running_mean"], sd[name + ".running_var"])
    y, cache, stats = op.bn_train_fwd(x, sd[name + ".weight"], sd[name + ".bias"], axes)
    t.push("bn", name, cache)
    t.stats[name] = stats
    return y


def _head(t, sd, x, train, use_attention):
    if use_attention:
        xa, a = op.attention_fwd(x, sd["attention.conv.weight"], sd["attention.conv.bias"])
        t.push("attn", x, a)
        x = xa
    t.push("avgpool", x.shape)
    pooled = op.avgpool_fwd(x)
    h = op.linear_fwd(pooled, sd["projection.0.weight"], sd["projection.0.bias"])
    t.push("linear", "projection.0", pooled)
    z = _bn(t, sd, "projection.1", h, train, (0,))
    e, ncache = op.normalize_fwd(z)
    t.push("normalize", ncache)
    return e


def _backward(t, sd, de):
    grads = {}
    g = de
    for rec in reversed(t.ops):
        kind = rec[0]
        if kind == "normalize":
            g = op.normalize_bwd(g, rec[1])
        elif kind == "bn":
            g, dgam, dbet = op.bn_train_bwd(g, rec[2])
            grads[rec[1] + ".weight"] = dgam
            grads[rec[1] + ".bias"] = dbet
        elif kind == "linear":
            pooled = rec[2]
            w = sd[rec[1] + ".weight"]
            g, dw, db = op.linear_bwd(g, pooled, w)
            grads[rec[1] + ".weight"] = dw
            grads[rec[1] + ".bias"] = db
        elif kind == "avgpool":
            g = op.avgpool_bwd(g, rec[1])
        elif kind == "attn":
            x, a = rec[1], rec[2]
            g, dwa, dba = op.attention_bwd(g, x, a, sd["attention.conv.weight"])
            grads["attention.conv.weight"] = dwa
            grads["attention.conv.bias"] = dba
        elif kind == "relu":
            g = op.relu_bwd(g, rec[1])
        elif kind == "pool":
            g = op.maxpool_bwd(g, rec[1])
        elif kind == "drop":
            if rec[1] is not None:
                g = g * rec[1][:, :, None, None]
        elif kind == "conv":
            name, x, stride, pad = rec[1:]
            need_dx = not (name in ("conv_blocks.0.0", "init_conv.0"))
            dx, dw, db = op.conv2d_bwd(x, sd[name + ".weight"], g, stride, pad, need_dx)
            grads[name + ".weight"] = dw
            grads[name + ".bias"] = db
            g = dx
        elif kind == "res_out":         # out = relu(z2 + sc): same grad into both branches
            g = op.relu_bwd(g, rec[1])
        elif kind == "shortcut":        # shortcut branch backward; main branch keeps g
            box, ops = rec[1], rec[2]
            if ops:
                sub = _Tape()
                sub.ops = ops
                gsx, sg = _backward(sub, sd, g)
                grads.update(sg)
            else:
                gsx = g
            box["g"] = gsx
        elif kind == "res_in":          # block input: add the shortcut-branch gradient
            g = g + rec[1]["g"]
    return g, grads


# ----------------------------------------------------------------------------- cnn_small
def small_forward(sd, x, train=True, masks=None, use_attention=None):
    """PhonemeNet.forward (phoneme_cnn.py:98-126)."""
    sd = _f64(sd)
    if use_attention is None:
        use_attention = "attention.conv.weight" in sd
    t = _Tape()
    h = np.asarray(x, dtype=np.float64)
    for blk in range(3):
        pre = f"conv_blocks.{blk}."
        for ci, bi in ((0, 1), (3, 4)):
            h = _conv(t, sd, pre + str(ci), h, 1, 1)
            h = _bn(t, sd, pre + str(bi), h, train, (0, 2, 3))
            h = op.relu_fwd(h)
            t.push("relu", h)
        if blk < 2:
            h, pc = op.maxpool_fwd(h, 2, 2, 0)
            t.push("pool", pc)
        m = None if (masks is None or not train) else np.asarray(masks[blk], dtype=np.float64)
        h = op.dropout2d(h, m)
        t.push("drop", m)
    e = _head(t, sd, h, train, use_attention)
    return e, t


# ----------------------------------------------------------------------------- cnn_deep
def deep_forward(sd, x, train=True, masks=None, use_attention=None):
    """PhonemeNetDeep.forward (phoneme_cnn.py:274-304) with ResidualBlock (:146-184)."""
    sd = _f64(sd)
    if use_attention is None:
        use_attention = "attention.conv.weight" in sd
    t = _Tape()
    h = np.asarray(x, dtype=np.float64)
    h = _conv(t, sd, "init_conv.0", h, 1, 3)
    h = _bn(t, sd, "init_conv.1", h, train, (0, 2, 3))
    h = op.relu_fwd(h)
    t.push("relu", h)
    h, pc = op.maxpool_fwd(h, 3, 2, 1)
    t.push("pool", pc)
    nblk = 0
    while f"conv_blocks.{nblk}.conv1.weight" in sd:
        nblk += 1
    for i in range(nblk):
        pre = f"conv_blocks.{i}."
        stride = 1 if i == 0 else 2
        xin = h
        box = {}
        # shortcut branch on its own tape
        st = _Tape()
        if pre + "shortcut.0.weight" in sd:
            s = _conv(st, sd, pre + "shortcut.0", xin, stride, 0)
            s = _bn(st, sd, pre + "shortcut.1", s, train, (0, 2, 3))
            t.stats.update(st.stats)
        else:
            s = xin
        t.push("res_in", box)
        a = _conv(t, sd, pre + "conv1", xin, stride, 1)
        a = _bn(t, sd, pre + "bn1", a, train, (0, 2, 3))
        a = op.relu_fwd(a)
        t.push("relu", a)
        m = None if (masks is None or not train) else np.asarray(masks[i], dtype=np.float64)
        a = op.dropout2d(a, m)
        t.push("drop", m)
        a = _conv(t, sd, pre + "conv2", a, 1, 1)
        a = _bn(t, sd, pre + "bn2", a, train, (0, 2, 3))
        t.push("shortcut", box, st.ops)
        h = op.relu_fwd(a + s)
        t.push("res_out", h)
    e = _head(t, sd, h, train, use_attention)
    return e, t


def forward(sd, x, train=True, masks=None):
    return (deep_forward if is_deep(sd) else small_forward)(sd, x, train, masks)


def backward(sd, tape, de):
    _, grads = _backward(tape, _f64(sd), de)
    return grads


# ----------------------------------------------------------------------------- train step
class AdamState:
    def __init__(self):
        self.m, self.v, self.step = {}, {}, 0


def train_step(sd, x, labels, masks, temperature=0.15, base_temperature=0.07, lr=3e-4,
               weight_decay=1e-4, opt=None):
    """One ContrastiveTrainer._train_epoch iteration (trainer.py:137-152): forward, SupCon,
    backward, Adam.step.  Returns (emb, loss, grads, new_state_dict)."""
    sd = _f64(sd)
    e, tape = forward(sd, x, True, masks)
    loss, de = op.supcon_fwd_bwd(e, labels, None, temperature, base_temperature)
    grads = backward(sd, tape, de)
    new = dict(sd)
    for name, st in tape.stats.items():
        rm, rv = op.bn_update_running(sd[name + ".running_mean"], sd[name + ".running_var"], st)
        new[name + ".running_mean"] = rm
        new[name + ".running_var"] = rv
        new[name + ".num_batches_tracked"] = np.asarray(sd[name + ".num_batches_tracked"]) + 1
    opt = opt or AdamState()
    opt.step += 1
    for k in param_names(sd):
        m = opt.m.get(k, np.zeros_like(sd[k]))
        v = opt.v.get(k, np.zeros_like(sd[k]))
        p, m, v = op.adam_step(sd[k], grads[k], m, v, opt.step, lr=lr, weight_decay=weight_decay)
        new[k], opt.m[k], opt.v[k] = p, m, v
    return e, loss, grads, new, opt
