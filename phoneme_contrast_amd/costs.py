"""Algorithmic cost model of the train step:
FLOPs and HBM bytes per kernel launch and per step for cnn_small and cnn_deep, and the MI355X
peaks they are priced against.  Used by bench.py (roofline of the dominant kernel, step
fractions) and by ContrastiveTrainer's perf.json."""

FP32_PEAK_TFLOPS = 157.3     # MI355X vector == matrix fp32 (MI355X_MICROARCH.md)
BF16_PEAK_TFLOPS = 2500.0    # dense bf16 MFMA (MI355X_MICROARCH.md: ~2.5 PF dense, no sparsity)
HBM_PEAK_GBS = 8000.0        # HBM3E spec
DEEP_DIMS = [64, 128, 256, 512]


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
    # pooled gradient hand-over (net.hip Layer::pd, even widths): layer 3 / 5's data gradient writes the
    # routed gradient at the pooled resolution and layer 2 / 4's weight gradient rebuilds dz from it and the
    # window selection (4 + 1 bytes per pooled element instead of 4 per full-resolution element)
    pd = {2: T % 4 == 0 and F % 2 == 0, 4: (T // 2) % 4 == 0 and (F // 2) % 2 == 0}
    for l, (ci, co, h, w) in L.items():
        macs = B * h * w * co * ci * 9
        sh, sw = src_res[l]
        y_out = 4 * B * co * h * w
        x_in = 4 * B * ci * sh * sw
        if l == 1:
            out["conv1_fwd_L1"] = (2 * macs, 4 * B * F * T + y_out)
            # (round 4: y1 is recomputed from the input window, not read: dz1 + x)
            out["wgrad_L1"] = (2 * macs, y_out + 4 * B * F * T)
            continue
        out[f"conv_fwd_L{l}"] = (2 * macs, x_in + y_out)
        # dgrad: reads dy_l (materialised by the weight gradient), the producer's values for its ReLU /
        # BN-backward epilogue -- y_{l-1} at full resolution, or behind a MaxPool2 the forward's recorded
        # selection (y at the selected element + its index: 5 bytes per pooled input, EPI_BWD_POOLSEL) --
        # and writes dz_{l-1} at full resolution
        prod = 5 * B * ci * h * w if (sh, sw) != (h, w) else x_in
        dz_prev = B * ci * h * w * 4 if pd.get(l - 1) else x_in  # pooled hand-over: dz_{l-1} at h x w
        out[f"conv_dgrad_L{l}"] = (2 * macs, y_out + prod + dz_prev)
        # wgrad: reads dz_l (or its pooled form + selection), y_l and the forward input source
        dz_in = y_out * 5 // 16 if pd.get(l) else y_out
        out[f"wgrad_L{l}"] = (2 * macs, dz_in + y_out + x_in)
        if l == 2:  # the fused layer-2 backward (wgbd_wino.hip): both GEMMs; dz2, y2, y1 read, dz1 written
            out["wgbd_L2"] = (4 * macs, dz_in + y_out + 2 * x_in)
    # elementwise / head passes (bytes: each tensor read once, each output written once)
    H1, W1, H3, W3, H5, W5 = F, T, F // 2, T // 2, F // 4, T // 4
    # (+ the recorded selection for the pooled data gradient: y at the selected element, its index)
    out["bn_relu_pool_L3"] = (0, B * 32 * (4 * H1 * W1 + 9 * H3 * W3))
    out["bn_relu_pool_L5"] = (0, B * 64 * (4 * H3 * W3 + 9 * H5 * W5))
    out["head_pool_fwd"] = (4 * B * 128 * H5 * W5, 4 * B * (128 * H5 * W5 + 128 + H5 * W5))
    out["head_pool_bwd"] = (6 * B * 128 * H5 * W5, 4 * B * (2 * 128 * H5 * W5 + 128 + H5 * W5))
    out["proj_fwd"] = (2 * B * 128 * D, 4 * B * (128 + 2 * D))
    out["proj_bwd"] = (4 * B * 128 * D, 4 * B * (2 * 128 + 3 * D))
    return out


def wino_tile_fraction(H, W):
    """Multiplies Winograd F(2x2,3x3) executes per direct-conv multiply on an H x W output: 16 per 2 x 2
    tile, ceil(H / 2) x ceil(W / 2) tiles, against 9 per output (4/9 at even H and W; 5 x 25 -> 0.555)."""
    return 16.0 * ((H + 1) // 2) * ((W + 1) // 2) / (9.0 * H * W)


def wgrad_wino_routed(H, W, cin, cout):
    """Whether the 3x3 weight gradient runs on the Winograd kernel: csrc/wgrad_wino.hip
    wgrad_wino_geometry() restated (staging vector 4 / 2 / 1 floats; odd widths only where the 2 x 2 tiles'
    outputs are >= 75 % real; strips of <= 50 tiles; 80 KB of LDS)."""
    if cin % 32 or cout % 32 or H < 1 or W < 4:
        return False
    V = 4 if W % 4 == 0 else 2 if W % 2 == 0 else 1
    TC = (W + 1) // 2
    if V == 1 and H * W < 0.75 * 4.0 * ((H + 1) // 2) * TC:
        return False
    nseg = -(-TC // 50)
    S = -(-TC // nseg)
    if nseg > 1:
        S = (S + 1) & ~1
    nseg = -(-TC // S)
    Ks = (S + 1) // 2
    nd, kmax = 2 * S // V, (2 * S + 1 + V - 1) // V
    nx = kmax + 1
    if (2 * S) % V or 2 * nd > 64 or 2 * nx > 64:
        return False

    def odd2(n):  # smallest m >= n with m = 2 * odd
        while n % 4 != 2:
            n += 1
        return n
    XCS = odd2(max(V * kmax + 1, 4 * Ks + 2, 2 * S + 5))
    DCS = odd2(4 * Ks)
    return (4 + 128 * XCS + 64 * DCS) * 4 <= 80 * 1024


def executed_fraction(label, T, F=40):
    """Multiplies executed per algorithmic (direct-conv) multiply for cnn_small's kernels: the 3x3
    forward / data-gradient convs run Winograd F(2x2,3x3) at W >= 31 (conv_wino.hip), the 3x3
    weight gradients where wgrad_wino_routed() (wgrad_wino.hip), the fused layer-2 backward (wgbd_wino.hip)
    on both; a Winograd kernel executes wino_tile_fraction() of the direct multiplies (partial tiles at odd
    sizes count whole).  Padding MFMAs a kernel runs beyond its tiles (wgbd's partial 16-tile groups) are not
    counted: the MOPS counter includes them."""
    shape = {2: (F, T, 32, 32), 3: (F // 2, T // 2, 32, 64), 4: (F // 2, T // 2, 64, 64),
             5: (F // 4, T // 4, 64, 128), 6: (F // 4, T // 4, 128, 128)}
    for pre in ("conv_fwd_L", "conv_dgrad_L"):
        if label.startswith(pre):
            H, W, _, _ = shape.get(int(label[len(pre):]), (0, 0, 0, 0))
            return wino_tile_fraction(H, W) if W >= 31 else 1.0
    if label.startswith("wgrad_L") and label[7:].isdigit() and int(label[7:]) >= 2:
        H, W, ci, co = shape[int(label[7:])]
        return wino_tile_fraction(H, W) if wgrad_wino_routed(H, W, ci, co) else 1.0
    if label == "wgbd_L2":  # fused layer-2 backward: both gradients on Winograd F(2x2,3x3)
        return wino_tile_fraction(F, T)
    return 1.0


def deep_executed_fraction(label, F, T, bf16=False, h=DEEP_DIMS):
    """Multiplies executed per algorithmic multiply for cnn_deep's kernels (deep.hip routing): in fp32
    the stride-1 3x3 convs whose channel counts fit the cnn_small engines (block 0 conv1, every conv2)
    run forward / data gradient on Winograd F(2x2,3x3) (conv_wino.hip: rows >= 31 columns, and the
    batch-spanning units below that) and the weight gradient on wgrad_wino.hip where wgrad_wino_routed();
    a Winograd kernel executes wino_tile_fraction() of the direct multiplies (5 x 25: 0.555, 3 x 13: 0.635);
    the stem, the stride-2 convs, the 1x1 shortcuts and every bf16 conv are direct."""
    if bf16:
        return 1.0
    routed = {}
    for fl, wl, dl, ci, co, k, s, IH, IW, OH, OW in deep_convs(F, T, h):
        fits = (co == 32 or co % 64 == 0) and (ci == 32 or ci % 64 == 0)
        if k == 3 and s == 1 and fits:
            routed[fl] = routed[dl] = wino_tile_fraction(OH, OW)
            routed[wl] = wino_tile_fraction(OH, OW) if wgrad_wino_routed(OH, OW, ci, co) else 1.0
    return routed.get(label, 1.0)


def executed_step_flops(B, F, T, D=128, deep=False, bf16=False):
    """FLOPs the step executes: the algorithmic step FLOPs with every Winograd kernel's convolution
    counted at the multiplies it performs (16 per 2x2 outputs instead of 36)."""
    if deep:
        total, _ = deep_step_cost(B, F, T, D, e=2 if bf16 else 4)
        costs = deep_kernel_costs(B, F, T, bf16, D)
        frac = lambda lab: deep_executed_fraction(lab, F, T, bf16)  # noqa: E731
        labels = [lab for c in deep_convs(F, T) for lab in c[:3] if lab]
    else:
        total, _ = step_cost(B, F, T, D)
        costs = kernel_costs(B, F, T, D)
        frac = lambda lab: executed_fraction(lab, T, F)  # noqa: E731
        # (at even widths layer 2's data gradient and weight gradient run as one kernel, wgbd_L2, with the
        # same executed fraction as the two it replaces)
        labels = [f"{p}{l}" for l in range(2, 7) for p in ("conv_fwd_L", "conv_dgrad_L", "wgrad_L")]
    saved = sum(costs[lab][0] * (1.0 - frac(lab)) for lab in labels if lab in costs)
    return int(total - saved)


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
        # bf16 (residual): the outputs of blocks 0-2 leave a byte ReLU mask instead of the float32 plane
        m8 = bf16 and i < 3
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


def deep_step_cost(B, F, T, D=128, e=4, h=DEEP_DIMS, nparams=4968833):
    """SURVEY 8(d)'s cnn_deep model: input read twice, every conv output written / read / re-read /
    gradient written / read (5 passes), the same for the init max-pool output and every block
    output; + 40 B per parameter and 12 B*D for SupCon (122.37 GB / step at B = 4096, T = 200)."""
    flops, act = 0, e * 2 * B * F * T
    for fl, wl, dl, ci, co, k, s, IH, IW, OH, OW in deep_convs(F, T, h):
        macs = B * OH * OW * co * ci * k * k
        flops += 2 * macs * (3 if dl else 2)
        act += e * 5 * B * co * OH * OW
    H, W = (F - 1) // 2 + 1, (T - 1) // 2 + 1
    act += e * 5 * B * h[0] * H * W  # init max-pool output
    for i, co in enumerate(h):
        s = 1 if i == 0 else 2
        H, W = (H - 1) // s + 1, (W - 1) // s + 1
        act += e * 5 * B * co * H * W        # block output
    flops += 4 * B * B * D + 3 * 2 * B * h[-1] * D
    return flops, act + 40 * nparams + 12 * B * D


def small_nparams(D=128, use_attention=True):
    """Parameter count of cnn_small (PhonemeNet, reference src/models/phoneme_cnn.py:31-80): convs
    1->32->32, 32->64->64, 64->128->128 with BN, the 1x1 attention conv, Linear(128, D) + BN1d(D)."""
    n = 0
    for ci, co in ((1, 32), (32, 32), (32, 64), (64, 64), (64, 128), (128, 128)):
        n += co * ci * 9 + co + 2 * co
    if use_attention:
        n += 128 + 1
    return n + 128 * D + D + 2 * D


def step_cost(B, F, T, D=128, nparams=None):
    """Algorithmic FLOPs and bytes of one whole train step; nparams defaults
    to cnn_small's own count at this D (304,225 at D = 128 with attention)."""
    flops = 0
    act_bytes = 4 * 2 * B * F * T  # input read twice
    for l, ci, co, h, w in small_layers(B, F, T):
        macs = B * h * w * co * ci * 9
        flops += 2 * macs * (2 if l == 1 else 3)
        act_bytes += 4 * 5 * B * co * h * w
    flops += 4 * B * B * D + 3 * 2 * B * 128 * D
    params = small_nparams(D) if nparams is None else nparams
    return flops, act_bytes + 40 * params + 12 * B * D


def model_step_cost(model, B, F, T):
    """(FLOPs, bytes, peak TFLOP/s, executed FLOPs) of one train step of `model` (a PhonemeNet /
    PhonemeNetDeep) at per-rank batch B and input [B, 1, F, T] under this cost model, or None for
    other models.  Executed FLOPs count the Winograd kernels at the multiplies they perform."""
    name = type(model).__name__
    D = getattr(model, "embedding_dim", 128)
    if name == "PhonemeNet":
        fl, by = step_cost(B, F, T, D, nparams=sum(p.numel() for p in model.parameters()))
        return fl, by, FP32_PEAK_TFLOPS, fl - (step_cost(B, F, T, D)[0] - executed_step_flops(B, F, T, D))
    if name == "PhonemeNetDeep":
        bf16 = getattr(model, "precision", "fp32") == "bf16"
        n = sum(p.numel() for p in model.parameters())
        h = list(model.hidden_dims)
        fl, by = deep_step_cost(B, F, T, D, e=2 if bf16 else 4, h=h, nparams=n)
        xfl = fl if (bf16 or h != DEEP_DIMS) else executed_step_flops(B, F, T, D, deep=True)
        return fl, by, BF16_PEAK_TFLOPS if bf16 else FP32_PEAK_TFLOPS, xfl
    return None
