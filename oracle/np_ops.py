"""float64 numpy restatement of the ops on the phoneme-contrast hot path (test oracle).

Every forward has a hand-derived backward; nothing here uses autograd.  Layout is the
reference's NCHW.  Citations are to /root/reference (read-only, not shipped).
"""
import numpy as np

EPS_BN = 1e-5          # nn.BatchNorm2d / BatchNorm1d default eps
MOMENTUM_BN = 0.1      # nn.BatchNorm default momentum


# ----------------------------------------------------------------------------- conv2d
def _windows(xp, kh, kw, stride, ho, wo):
    """[B,C,Hp,Wp] -> view [B,C,kh,kw,ho,wo] of the strided receptive fields."""
    b, c, _, _ = xp.shape
    sb, sc, sh, sw = xp.strides
    return np.lib.stride_tricks.as_strided(
        xp, shape=(b, c, kh, kw, ho, wo),
        strides=(sb, sc, sh, sw, sh * stride, sw * stride), writeable=False)


def conv2d_fwd(x, w, b, stride=1, pad=0):
    """nn.Conv2d forward (phoneme_cnn.py:36,39,47,50,58,61,135,159-161,212; cross-correlation)."""
    o, c, kh, kw = w.shape
    bsz, _, h, wd = x.shape
    ho = (h + 2 * pad - kh) // stride + 1
    wo = (wd + 2 * pad - kw) // stride + 1
    xp = np.pad(x, ((0, 0), (0, 0), (pad, pad), (pad, pad)))
    win = _windows(xp, kh, kw, stride, ho, wo)
    y = np.einsum("bcijhw,ocij->bohw", win, w, optimize=True)
    if b is not None:
        y = y + b[None, :, None, None]
    return y


def conv2d_bwd(x, w, dy, stride=1, pad=0, need_dx=True):
    """Gradients of conv2d_fwd: (dx, dw, db)."""
    o, c, kh, kw = w.shape
    bsz, _, h, wd = x.shape
    ho, wo = dy.shape[2], dy.shape[3]
    xp = np.pad(x, ((0, 0), (0, 0), (pad, pad), (pad, pad)))
    win = _windows(xp, kh, kw, stride, ho, wo)
    dw = np.einsum("bcijhw,bohw->ocij", win, dy, optimize=True)
    db = dy.sum(axis=(0, 2, 3))
    dx = None
    if need_dx:
        dxp = np.zeros_like(xp)
        for i in range(kh):
            for j in range(kw):
                contrib = np.einsum("bohw,oc->bchw", dy, w[:, :, i, j], optimize=True)
                dxp[:, :, i:i + stride * ho:stride, j:j + stride * wo:stride] += contrib
        dx = dxp[:, :, pad:pad + h, pad:pad + wd]
    return dx, dw, db


# ----------------------------------------------------------------------------- batchnorm
def bn_train_fwd(x, gamma, beta, axes):
    """Train-mode BatchNorm (batch statistics, biased variance for normalisation)."""
    mean = x.mean(axis=axes, keepdims=True)
    var = x.var(axis=axes, keepdims=True)
    invstd = 1.0 / np.sqrt(var + EPS_BN)
    xhat = (x - mean) * invstd
    shape = [1] * x.ndim
    shape[1] = -1
    y = xhat * gamma.reshape(shape) + beta.reshape(shape)
    n = x.size // x.shape[1]
    cache = (xhat, invstd, gamma.reshape(shape), axes)
    stats = (mean.reshape(-1), var.reshape(-1) * n / max(n - 1, 1))
    return y, cache, stats


def bn_train_bwd(dy, cache):
    xhat, invstd, g, axes = cache
    n = dy.size // dy.shape[1]
    dbeta = dy.sum(axis=axes)
    dgamma = (dy * xhat).sum(axis=axes)
    shape = [1] * dy.ndim
    shape[1] = -1
    dx = g * invstd * (dy - dbeta.reshape(shape) / n - xhat * dgamma.reshape(shape) / n)
    return dx, dgamma, dbeta


def bn_update_running(rm, rv, stats):
    """running = (1-m)*running + m*batch (unbiased var), torch BN semantics."""
    mean, var_unb = stats
    return (1 - MOMENTUM_BN) * rm + MOMENTUM_BN * mean, (1 - MOMENTUM_BN) * rv + MOMENTUM_BN * var_unb


def bn_eval(x, gamma, beta, rm, rv):
    shape = [1] * x.ndim
    shape[1] = -1
    return (x - rm.reshape(shape)) / np.sqrt(rv.reshape(shape) + EPS_BN) * gamma.reshape(shape) \
        + beta.reshape(shape)


# ----------------------------------------------------------------------------- relu / pool
def relu_fwd(x):
    return np.maximum(x, 0.0)


def relu_bwd(dy, out):
    # torch threshold_backward uses the ReLU output: grad where out > 0
    return dy * (out > 0)


def maxpool_fwd(x, k, s, p):
    """nn.MaxPool2d(k, s, p) (phoneme_cnn.py:42,53 with k=s=2,p=0; :215 with 3,2,1).
    Returns output and the flat argmax (first maximum in window scan order)."""
    bsz, c, h, w = x.shape
    ho = (h + 2 * p - k) // s + 1
    wo = (w + 2 * p - k) // s + 1
    xp = np.pad(x, ((0, 0), (0, 0), (p, p), (p, p)), constant_values=-np.inf)
    win = _windows(xp, k, k, s, ho, wo)                    # [B,C,k,k,ho,wo]
    flat = win.transpose(0, 1, 4, 5, 2, 3).reshape(bsz, c, ho, wo, k * k)
    arg = flat.argmax(axis=-1)
    y = np.take_along_axis(flat, arg[..., None], axis=-1)[..., 0]
    return y, (arg, x.shape, k, s, p)


def maxpool_bwd(dy, cache):
    arg, xshape, k, s, p = cache
    bsz, c, h, w = xshape
    ho, wo = dy.shape[2], dy.shape[3]
    dxp = np.zeros((bsz, c, h + 2 * p, w + 2 * p))
    ii = arg // k
    jj = arg % k
    hh = ii + s * np.arange(ho)[None, None, :, None]
    ww = jj + s * np.arange(wo)[None, None, None, :]
    bb = np.arange(bsz)[:, None, None, None]
    cc = np.arange(c)[None, :, None, None]
    np.add.at(dxp, (bb, cc, hh, ww), dy)
    return dxp[:, :, p:p + h, p:p + w]


# ----------------------------------------------------------------------------- dropout2d
def dropout2d(x, mask):
    """nn.Dropout2d with an injected per-(sample, channel) keep-scale (0 or 1/(1-p))."""
    if mask is None:
        return x
    return x * mask[:, :, None, None]


# ----------------------------------------------------------------------------- attention + pool
def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def attention_fwd(x, wa, ba):
    """SpatialAttention (phoneme_cnn.py:129-143): a = sigmoid(conv1x1(x)); y = x * a."""
    logit = np.einsum("bchw,c->bhw", x, wa.reshape(-1)) + ba.reshape(())
    a = sigmoid(logit)[:, None]
    return x * a, a


def attention_bwd(dy, x, a, wa):
    da = (dy * x).sum(axis=1, keepdims=True)
    dlogit = da * a * (1 - a)
    dx = dy * a + dlogit * wa.reshape(1, -1, 1, 1)
    dwa = np.einsum("bhw,bchw->c", dlogit[:, 0], x).reshape(wa.shape)
    dba = np.array([dlogit.sum()])
    return dx, dwa, dba


def avgpool_fwd(x):
    """AdaptiveAvgPool2d(1) + view (phoneme_cnn.py:74,116-117)."""
    return x.mean(axis=(2, 3))


def avgpool_bwd(dy, shape):
    b, c, h, w = shape
    return np.broadcast_to(dy[:, :, None, None] / (h * w), shape).copy()


# ----------------------------------------------------------------------------- head
def linear_fwd(x, w, b):
    return x @ w.T + b


def linear_bwd(dy, x, w):
    return dy @ w, dy.T @ x, dy.sum(axis=0)


def normalize_fwd(x, eps=1e-12):
    """F.normalize(p=2, dim=1) (phoneme_cnn.py:124): x / max(||x||, eps)."""
    n = np.sqrt((x * x).sum(axis=1, keepdims=True))
    d = np.maximum(n, eps)
    return x / d, (x, n, d, eps)


def normalize_bwd(dy, cache):
    x, n, d, eps = cache
    y = x / d
    live = (n > eps)
    # d(x/d)/dx = I/d - x x^T/(d n) * [n > eps]
    return dy / d - live * y * (dy * x).sum(axis=1, keepdims=True) / (d * np.where(live, n, 1.0))


# ----------------------------------------------------------------------------- SupCon
def supcon_fwd_bwd(f, labels=None, mask=None, temperature=0.07, base_temperature=0.07,
                   reduction="mean"):
    """SupervisedContrastiveLoss (losses.py:41-86) and its closed-form gradient dL/dF
    (SURVEY Appendix A).  For reduction='none' the returned gradient is that of loss.sum().
    Returns (loss, dF)."""
    f = np.asarray(f, dtype=np.float64)
    bsz = f.shape[0]
    if bsz == 1:
        raise ValueError("Batch size must be greater than 1 for contrastive loss")
    if mask is None:
        lab = np.asarray(labels).reshape(-1, 1)
        m = (lab == lab.T).astype(np.float64)
    else:
        m = np.asarray(mask, dtype=np.float64)
    lm = 1.0 - np.eye(bsz)
    m = m * lm
    s = f @ f.T
    logits = s / temperature
    z = logits - logits.max(axis=1, keepdims=True)        # row max includes the diagonal
    e = np.exp(z) * lm
    den = e.sum(axis=1, keepdims=True) + 1e-6             # eps inside the log
    log_prob = z - np.log(den)
    msum = m.sum(axis=1)
    p = np.where(msum == 0, 1.0, msum)
    mlpp = (m * log_prob).sum(axis=1) / p
    scale = temperature / base_temperature
    per = -scale * mlpp
    if reduction == "mean":
        loss, w = per.mean(), np.full(bsz, 1.0 / bsz)
    elif reduction == "sum":
        loss, w = per.sum(), np.ones(bsz)
    else:
        loss, w = per, np.ones(bsz)
    dz = -(scale * w / p)[:, None] * (m - msum[:, None] * e / den)
    g = dz / temperature
    df = (g + g.T) @ f
    return loss, df


def _pos_mask(bsz, labels, mask):
    if mask is None:
        lab = np.asarray(labels).reshape(-1, 1)
        return (lab == lab.T).astype(np.float64) * (1.0 - np.eye(bsz))
    return np.asarray(mask, dtype=np.float64) * (1.0 - np.eye(bsz))


def supcon_rows_fwd(f, labels, mask, row0, nrows, temperature=0.07, base_temperature=0.07,
                    reduction="mean"):
    """Anchor rows [row0, row0+nrows) of SupCon over the batch f [B, D] (the global-batch mode's
    per-rank forward, include/pcx.h pcx_supcon_forward_rows).  Returns (loss share, rowstats
    [nrows, 4] = (m_i, den_i, msum_i, loss_i)); the shares of a partition of [0, B) sum to the
    reference loss (losses.py:41-86) of the whole batch."""
    f = np.asarray(f, dtype=np.float64)
    bsz = f.shape[0]
    rows = np.arange(row0, row0 + nrows)
    m = _pos_mask(bsz, labels, mask)[rows]
    lm = np.ones((nrows, bsz))
    lm[np.arange(nrows), rows] = 0.0
    logits = f[rows] @ f.T / temperature
    mx = logits.max(axis=1)
    e = np.exp(logits - mx[:, None]) * lm
    den = e.sum(axis=1) + 1e-6
    msum = m.sum(axis=1)
    p = np.where(msum == 0, 1.0, msum)
    mlpp = (m * (logits - mx[:, None] - np.log(den)[:, None])).sum(axis=1) / p
    per = -(temperature / base_temperature) * mlpp
    share = {"mean": per.sum() / bsz, "sum": per.sum()}.get(reduction, per)
    return share, np.stack([mx, den, msum, per], axis=1)


def supcon_coef_rows(rowstats, grad_out, bsz, base_temperature=0.07, reduction="mean"):
    """Per-anchor gradient coefficients (a_i, b_i, m_i) of pcx_supcon_coef_rows:
    dLoss_i/dS_ij = a_i M_ij - b_i exp(S_ij/T - m_i) (j != i) with a_i = -w_i / (bT P_i),
    b_i = a_i msum_i / den_i and w_i the anchor's weight in the reduction."""
    mx, den, msum = rowstats[:, 0], rowstats[:, 1], rowstats[:, 2]
    g = np.asarray(grad_out, dtype=np.float64).reshape(-1)
    w = g if reduction == "none" else np.full(len(mx), g[0] / bsz if reduction == "mean" else g[0])
    a = -w / base_temperature / np.where(msum == 0, 1.0, msum)
    return np.stack([a, a * msum / den, mx], axis=1)


def supcon_rows_bwd(f, labels, mask, row0, nrows, coef_all, temperature=0.07):
    """dLoss/dF of rows [row0, row0+nrows) given every anchor's coefficients (pcx_supcon_backward_rows):
    dF_i = sum_j (H_ij + H_ji) F_j, H_ij = a_i M_ij - b_i exp(S_ij/T - m_i), j != i -- the
    anchor-side and column-side terms, so the ranges' results need no reduction."""
    f = np.asarray(f, dtype=np.float64)
    bsz = f.shape[0]
    m = _pos_mask(bsz, labels, mask)
    z = f @ f.T / temperature
    a, b, mx = coef_all[:, 0], coef_all[:, 1], coef_all[:, 2]
    h = a[:, None] * m - b[:, None] * np.exp(z - mx[:, None]) * (1.0 - np.eye(bsz))
    rows = slice(row0, row0 + nrows)
    return (h + h.T)[rows] @ f


def ntxent_fwd_bwd(f, labels, temperature=0.07, reduction="mean"):
    """NTXentLoss labelled branch (losses.py:101-151) == SupCon with base_temperature=T."""
    if labels is None:
        if f.shape[0] % 2 != 0:
            raise ValueError("Batch size must be even for NT-Xent loss without labels")
        raise NotImplementedError("NT-Xent without labels not implemented in this version")
    return supcon_fwd_bwd(f, labels, None, temperature, temperature, reduction)


# ----------------------------------------------------------------------------- Adam
def adam_step(p, g, m, v, step, lr=3e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
    """torch.optim.Adam (coupled L2, scripts/train.py:129-133): returns new (p, m, v).
    `step` is the 1-based step count after increment."""
    b1, b2 = betas
    g = g + weight_decay * p
    m = b1 * m + (1 - b1) * g
    v = b2 * v + (1 - b2) * g * g
    bc1 = 1 - b1 ** step
    bc2 = 1 - b2 ** step
    denom = np.sqrt(v) / np.sqrt(bc2) + eps
    p = p - (lr / bc1) * m / denom
    return p, m, v
