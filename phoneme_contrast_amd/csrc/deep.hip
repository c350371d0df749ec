// cnn_deep plan: PhonemeNetDeep forward / backward (reference src/models/phoneme_cnn.py:146-304).
//
//   stem   y0 = conv7x7(x) (pad 3)      a0 = MaxPool(3,2,1)(ReLU(BN0(y0)))            :211-216
//   block  y1 = conv3x3_s(a)   d1 = Dropout2d(ReLU(BN1(y1)))                          :174-176
//          y2 = conv3x3(d1)    sc = a | BNsc(conv1x1_s(a))                            :166-171,177-180
//          a' = ReLU(BN2(y2) + sc)                                                     :181
//   (use_residual = false, :230-243:  a' = Dropout2d(ReLU(BN2(conv(ReLU(BN1(conv_s(a))))))))
//   head   attention(512) -> mean -> Linear -> BN1d -> normalize (shared with cnn_small, head.hip)
//
// Raw conv outputs (bias excluded: every conv feeds a train-mode BN, so its bias only shifts the
// running mean) and the block outputs are kept in the workspace; BN statistics are reduced in
// float64 by the same finalisers as cnn_small.  Convolutions run on the general implicit-GEMM
// MFMA kernel (convg.hip); BN / ReLU / residual / dropout are elementwise passes.
#include <algorithm>
#include "plan.h"

namespace pcx {

struct DeepBlock {
    int cin, cout, stride, Hi, Wi, Ho, Wo;
    bool sc;                      // 1x1 conv + BN shortcut
    int pidx, bnidx, drop_idx;
    size_t y1, d1, y2, ysc, out;  // forward tensors
    size_t cf1, cf2, cfsc, cfb1, cfb2, cfbsc;
    size_t da;                    // gradient w.r.t. the block input
    // stride-1 3x3 convs routed to the cnn_small engines (conv_dma.hip forward / data gradient,
    // wgrad_w32.hip weight gradient) when their channel counts fit; conv1 of block 0 and conv2
    bool dma1, dma2, w32_1, w32_2;
    WgradArgs wg1, wg2;
    // ... whose weight gradient runs on the Winograd kernel (wgrad_wino.hip) where it applies (even W);
    // w32_* then stays set: the BN backward is applied in its staging and dy written by it too
    bool ww1, ww2;
    WinoWgradArgs wwa1, wwa2;
    int nblk1, nblk2;
    // precision "bf16" with channel counts the channel-last engine takes (convn.hip): padded NHWC
    // bf16 images of the block input (conv1, shortcut) and of d1 (conv2), kept for the backward
    bool cn;
    bool planar;                   // stride-2 data gradient through class-planar planes
    size_t an, d1n;
    size_t m8;                     // channel-last next block: the output's ReLU mask as bytes (no float32 out)
};

// narrow stride-1 images (5 x 25, 3 x 13) on the Winograd conv with batch-spanning units
// (PCX_AB_NO_WINO_SPAN: the direct LDS-DMA conv)
static bool wino_span_ok() {
    constexpr bool off = PCX_AB_NO_WINO_SPAN;
    return !off;
}

struct DeepPlan {
    bool residual;
    bool bf16;                     // every conv on convg_bf16 (bf16 operands, float32 accumulation)
    int h[4];
    int H0, W0, H1, W1;
    size_t y0, a0, cf0, cfb0, dz0, mparg;
    bool stem_fused;               // bf16 stem with y0 recomputed (no y0 plane; conv.hip stem_pool_kernel)
    size_t ysel;                   // fused stem: y0 at each window's selected tap
    size_t stemw;                  // bf16-rounded stem weights (precision "bf16")
    int stem_nblk, stem_rows, stem_ns, stem_srows;  // stem forward blocks / weight-gradient slices
    size_t wpk, identw;           // packed 3x3 weights of a routed conv; identity BN coefficients
    size_t wpk16;                 // packed GEMM weights of the current general-engine conv
    int cmax;
    DeepBlock blk[4];
    size_t g, dyA, dyB, dd, hdz;   // backward scratch
    size_t dyn1, dyn2;             // channel-last bf16 dy images (conv1 / conv2, shortcut)
    size_t partmp;                 // class-planar stride-2 data gradient (ConvGArgs::par_out), or 0
    size_t stat, wgp, ident;
    int ia, ip;                    // attention / projection parameter indices
    int bn_proj;
};

namespace {

int64_t planes(int B, int C, int H, int W) { return (int64_t)B * C * H * W; }

NhwcArgs nhwc_args(int op, int B, int C, int H, int W, const float* src, void* dst) {
    NhwcArgs a{};
    a.op = op;
    a.B = B; a.C = C; a.H = H; a.W = W;
    a.src = src;
    a.dst = dst;
    return a;
}

}  // namespace

int build_deep(Plan& p) {
    auto dp = std::make_shared<DeepPlan>();
    DeepPlan& d = *dp;
    const int B = p.B;
    d.residual = p.cfg.use_residual != 0;
    d.bf16 = p.cfg.conv_bf16 != 0;
    for (int i = 0; i < 4; ++i) {
        d.h[i] = p.cfg.hidden_dims[i];
        PCX_CHECK_ARG(d.h[i] >= 1 && d.h[i] <= 4096, "PhonemeNetDeep: hidden_dims[%d] = %d unsupported", i, d.h[i]);
    }
    PCX_CHECK_ARG(p.F >= 1 && p.T >= 1, "PhonemeNetDeep: empty input");
    d.H0 = p.F; d.W0 = p.T;
    d.H1 = (d.H0 - 1) / 2 + 1; d.W1 = (d.W0 - 1) / 2 + 1;
    const int C0 = d.h[0];
    // (blocks 0 and 1 on the channel-last engine: block 0's output activation reads the pooled residual)
    d.stem_fused = d.bf16 && stem_fused_ok(C0, d.H0, d.W0) && d.h[0] % 32 == 0 && d.h[1] % 32 == 0;
    d.y0 = d.stem_fused ? 0 : p.carve("y0", planes(B, C0, d.H0, d.W0) * 4);
    d.dz0 = p.carve("dz0", planes(B, C0, d.H0, d.W0) * (d.stem_fused ? 2 : 4));  // fused: bf16
    d.a0 = p.carve("a0", planes(B, C0, d.H1, d.W1) * 4);
    d.mparg = p.carve("maxpool_arg", planes(B, C0, d.H1, d.W1));  // first-max tap per window (uint8)
    d.ysel = d.stem_fused ? p.carve("ysel", planes(B, C0, d.H1, d.W1) * 4) : 0;
    d.cf0 = p.carve("cf0", C0 * 16);
    d.cfb0 = p.carve("cfb0", C0 * 16);
    int pidx = 4, bnidx = 1, cin = C0, H = d.H1, W = d.W1;
    size_t gmax = 0, stat = 0, wg = 0, dynmax = 0, partmax = 0;
    auto wg_need = [&](int ci, int co, int k, int oh, int ow) {
        ConvGArgs a{};
        a.B = B; a.cin = ci; a.cout = co; a.KH = a.KW = k; a.OH = oh; a.OW = ow;
        int64_t ks;
        int ns = convg_nslice(a, &ks);
        wg = std::max(wg, (size_t)ns * co * ci * k * k);
    };
    auto stat_need = [&](int C) {
        int bps;
        int ns = chan_slices(B, C, &bps);
        stat = std::max(stat, (size_t)3 * C * ns + ns);
    };
    // the 7x7 stem runs on its own direct kernels (conv.hip): forward partials, gradient slices
    d.stem_nblk = stem_nblk(B, d.H0, &d.stem_rows);
    d.stem_ns = stem_wgrad_nslice(B, d.H0, &d.stem_srows,
                                  d.stem_fused || stem_wgrad_mfma_ok(d.h[0], d.H0, d.W0));
    stat = std::max(stat, (size_t)3 * C0 * d.stem_nblk + d.stem_nblk);
    wg = std::max(wg, (size_t)d.stem_ns * C0 * 49);
    d.stemw = p.carve("stem_w16", (size_t)C0 * 49 * 4);
    size_t wpk = 0;
    int cmax = 0;
    for (int i = 0; i < 4; ++i) cmax = std::max(cmax, d.h[i]);
    const bool route = !d.bf16;  // fp32: stride-1 3x3 convs on the LDS-DMA / 32x32 engines
    // a stride-1 3x3 conv cin -> cout at HxW on the DMA conv (fwd, dgrad) and the 32x32 wgrad
    auto plan_routed = [&](int ci, int co, int h, int w, bool* fwd, bool* w32, WgradArgs* wga, int* nblk,
                           bool* ww, WinoWgradArgs* wwa) {
        *fwd = route && (co == 32 || co % 64 == 0) && (ci == 32 || ci % 64 == 0) && ci % 2 == 0;
        // the Winograd weight gradient wherever its geometry takes the shape (even widths; odd widths past its
        // tile-coverage gate: 5 x 25, not 3 x 13); else the pixel-stream kernel from 50 columns
        // up (narrower rows waste its 8-column stream granule: the 32x32 row-window kernel takes them)
        *ww = route && wgrad_wino_geometry(B, h, w, ci, co, wwa);
        if (*ww) wg = std::max(wg, (size_t)wwa->nslice * co * ci * 16);
        *w32 = *ww || (route && (w >= 50 ? wgrad_s_geometry(B, h, w, ci, co, wga) : wgrad_w32_geometry(B, h, w, ci, co, wga)));
        *nblk = 0;
        if (*fwd) {
            // the Winograd conv takes the layers whose rows are >= 31 columns wide (its own tile blocks) and
            // the narrow ones it can span (5 x 25 / 3 x 13: units over rows and samples)
            *nblk = (int)std::max({conv3x3_nblk(B, h, w, co), conv3x3_nblk(B, h, w, ci), wino_nblk(B, h, w, ci, co),
                                   wino_nblk(B, h, w, co, ci)});
            stat = std::max(stat, (size_t)2 * std::max(ci, co) * (*nblk) + *nblk);
            wpk = std::max(wpk, (size_t)16 * ci * co);
        }
        if (*w32 && !*ww) wg = std::max(wg, (size_t)wga->nslice * co * ci * 9);
    };
    for (int i = 0; i < 4; ++i) {
        DeepBlock& k = d.blk[i];
        k.cin = cin; k.cout = d.h[i]; k.stride = i == 0 ? 1 : 2;
        k.Hi = H; k.Wi = W;
        k.Ho = (H - 1) / k.stride + 1; k.Wo = (W - 1) / k.stride + 1;
        k.sc = d.residual && (k.stride != 1 || k.cin != k.cout);
        k.pidx = pidx; k.bnidx = bnidx; k.drop_idx = i;
        pidx += 8 + (k.sc ? 4 : 0);
        bnidx += 2 + (k.sc ? 1 : 0);
        const size_t no = (size_t)planes(B, k.cout, k.Ho, k.Wo) * 4;
        char nm[24];
        snprintf(nm, sizeof nm, "b%d_y1", i); k.y1 = p.carve(nm, no);
        snprintf(nm, sizeof nm, "b%d_d1", i); k.d1 = p.carve(nm, no);
        snprintf(nm, sizeof nm, "b%d_y2", i); k.y2 = p.carve(nm, no);
        snprintf(nm, sizeof nm, "b%d_out", i); k.out = p.carve(nm, no);
        k.ysc = k.sc ? p.carve("ysc", no) : 0;
        snprintf(nm, sizeof nm, "b%d_da", i);
        k.da = p.carve(nm, (size_t)planes(B, k.cin, k.Hi, k.Wi) * 4);
        k.cf1 = p.carve("cf", k.cout * 16); k.cf2 = p.carve("cf", k.cout * 16);
        k.cfb1 = p.carve("cf", k.cout * 16); k.cfb2 = p.carve("cf", k.cout * 16);
        k.cfsc = p.carve("cf", k.cout * 16); k.cfbsc = p.carve("cf", k.cout * 16);
        gmax = std::max(gmax, no);
        stat_need(k.cout);
        wg_need(k.cin, k.cout, 3, k.Ho, k.Wo);
        wg_need(k.cout, k.cout, 3, k.Ho, k.Wo);
        if (k.sc) wg_need(k.cin, k.cout, 1, k.Ho, k.Wo);
        k.cn = d.bf16 && k.cin % 32 == 0 && k.cout % 32 == 0;
        k.planar = (k.cn || !d.bf16) && k.stride == 2 && (int64_t)planes(B, k.cin, k.Hi, k.Wi) < ((int64_t)1 << 31);
        if (k.planar) partmax = std::max(partmax, (size_t)planes(B, k.cin, k.Hi, k.Wi) * 4);
        k.an = k.d1n = k.m8 = 0;
        if (k.cn) {
            // the channel-last forward writes BN partials per 128-pixel tile (conv1, conv2, shortcut)
            const size_t nt = (size_t)convn_tile_bound(B, k.Ho, k.Wo);
            stat = std::max(stat, (size_t)2 * k.cout * nt + nt);
            k.an = p.carve("nhwc_a", nhwc_bytes(B, k.cin, k.Hi, k.Wi));
            k.d1n = p.carve("nhwc_d1", nhwc_bytes(B, k.cout, k.Ho, k.Wo));
            dynmax = std::max(dynmax, nhwc_bytes(B, k.cout, k.Ho, k.Wo));
        }
        k.dma1 = k.w32_1 = k.ww1 = false;
        k.nblk1 = 0;
        if (k.stride == 1) plan_routed(k.cin, k.cout, k.Ho, k.Wo, &k.dma1, &k.w32_1, &k.wg1, &k.nblk1, &k.ww1, &k.wwa1);
        plan_routed(k.cout, k.cout, k.Ho, k.Wo, &k.dma2, &k.w32_2, &k.wg2, &k.nblk2, &k.ww2, &k.wwa2);
        cin = k.cout; H = k.Ho; W = k.Wo;
    }
    // block outputs read only as a ReLU mask (the next block reads its NHWC image): bytes, at any width.
    // (Round 3 gated this on even widths after wrong forwards at T = 200 block 2 / T = 100 block 1 of
    // reduced-width nets.  The cause: in those nets block i is not channel-last but block i + 1 is, and
    // block i + 1's forward re-copied its NHWC input from block i's float32 output -- unwritten under the
    // byte mask -- over the image block i's activation had just written.  The even-width gate only
    // happened to exclude those cases.  The copy now runs only where nothing wrote the image (block 0
    // without the fused stem), and the forward / backward hand nullptr, never the unwritten plane, to
    // every consumer of a byte-masked output: the conv / shortcut GEMMs then must take the NHWC image.)
    for (int i = 0; i < 3; ++i)
        if (d.residual && d.blk[i + 1].cn)
            d.blk[i].m8 = p.carve("relu_mask8", (size_t)planes(B, d.blk[i].cout, d.blk[i].Ho, d.blk[i].Wo));
    d.g = p.carve("g", gmax);
    d.dyA = p.carve("dyA", gmax);
    d.dyB = p.carve("dyB", gmax);
    d.dd = p.carve("dd", gmax);
    d.partmp = partmax ? p.carve("par_planes", partmax) : 0;
    d.dyn1 = dynmax ? p.carve("nhwc_dy1", dynmax) : 0;
    d.dyn2 = dynmax ? p.carve("nhwc_dy2", dynmax) : 0;
    const int C4 = d.h[3];
    p.C6 = C4;
    p.P6 = H * W;
    d.hdz = p.carve("hdz", (size_t)planes(B, C4, H, W) * 4);
    stat = std::max(stat, (size_t)2 * C4 * B);
    if (d.stem_fused) stat = std::max(stat, (size_t)2 * C0 * B);  // stem_pool_bwd partials [C0][B] x 2
    d.stat = p.carve("stat_part", stat * 4);
    // stride-1 Winograd convs take their units from a per-XCD queue (PCX_AB_NO_WINO_QUEUE: static order)
    p.wq = PCX_AB_NO_WINO_QUEUE ? 0 : p.carve("wino_queue", WINO_QUEUE_INTS * 4);
    d.wgp = p.carve("wg_part", wg * 4);
    d.ident = p.carve("ident", (size_t)C4 * 16);
    d.identw = p.carve("identw", (size_t)cmax * 16);
    d.cmax = cmax;
    d.wpk = p.carve("wpack", std::max<size_t>(wpk, 1) * 4);
    {  // packed GEMM weights of the general engine (fp32 or bf16 rows)
        auto need = [&](int mode, int ci, int co, int kk) {
            return d.bf16 ? convg_bf16_wpack_bytes(mode, ci, co, kk) : convg_wpack_bytes(mode, ci, co, kk);
        };
        size_t w16 = need(0, 1, C0, 7);
        for (int i = 0; i < 4; ++i) {
            const DeepBlock& k = d.blk[i];
            for (int mode = 0; mode < 2; ++mode) {
                w16 = std::max(w16, need(mode, k.cin, k.cout, 3));
                w16 = std::max(w16, need(mode, k.cout, k.cout, 3));
                if (k.sc) w16 = std::max(w16, need(mode, k.cin, k.cout, 1));
            }
        }
        d.wpk16 = p.carve("wpack_g", w16);
    }
    d.ia = pidx;
    d.ip = pidx + (p.cfg.use_attention ? 2 : 0);
    d.bn_proj = bnidx;
    const int D = p.D, K = C4;
    p.pooled = p.carve("pooled", (size_t)B * K * 4);
    p.att = p.carve("att", (size_t)B * p.P6 * 4);
    p.h = p.carve("h", (size_t)B * D * 4);
    p.cfp = p.carve("cfp", (size_t)D * 16);
    p.cfpb = p.carve("cfpb", (size_t)D * 16);
    p.norm = p.carve("norm", (size_t)B * 4);
    p.dzp = p.carve("dzp", (size_t)B * D * 4);
    p.dh = p.carve("dh", (size_t)B * D * 4);
    p.dpooled = p.carve("dpooled", (size_t)B * K * 4);
    p.proj_part = p.carve("proj_part", proj_part_floats(B, D, K) * 4);
    p.wt = p.carve("wt", (size_t)K * D * 4);
    p.hp_dwa = p.carve("hp_dwa", (size_t)K * B * 4);
    p.hp_dba = p.carve("hp_dba", (size_t)B * 4);
    p.nparams = d.ip + 4;
    // backward completion points: projection, attention, blocks 3..0, stem
    p.stages = {d.ip};
    if (p.cfg.use_attention) p.stages.push_back(d.ia);
    for (int i = 3; i >= 0; --i) p.stages.push_back(d.blk[i].pidx);
    p.stages.push_back(0);
    p.nbn = bnidx + 1;
    p.ndrop = 4;
    for (int i = 0; i < 4; ++i) p.drop_ch[i] = d.h[i];
    p.deep = dp;
    return PCX_OK;
}

namespace {

struct Ctx {
    const Plan& p;
    const DeepPlan& d;
    void* ws;
    hipStream_t s;
    template <class T>
    T* w(size_t off) const { return at<T>(ws, off); }
};

// float32 output plane of block i, or nullptr when only its byte ReLU mask (and the next block's NHWC
// image) is stored: the plane is then never written, and no consumer may be handed it
const float* block_out(const Ctx& c, int i) {
    const DeepBlock& k = c.d.blk[i];
    return k.m8 ? nullptr : c.w<float>(k.out);
}

// forward conv (raw output, no bias) + train-mode statistics + BN finalise -> cf
int conv_bn_fwd(const Ctx& c, const char* label, int layer, const float* x, int cin, int IH, int IW, int k, int stride,
                int pad, const float* wgt, float* y, int cout, int OH, int OW, const float* gamma, const float* beta,
                const float* bias, float* rmean, float* rvar, int64_t* nbt, int train, float4* cf, int dma_nblk = 0,
                const void* xn = nullptr) {
    PCX_CHECK_ARG(x || xn, "deep plan: %s of layer %d has no input (float32 plane or NHWC image)", label, layer);
    float* part = c.w<float>(c.d.stat);
    int ns = 1;
    BnFwdArgs f{};
    f.C = cout;
    if (dma_nblk) {  // stride-1 3x3 on the LDS-DMA conv: its epilogue writes the BN partials
        float* wp = c.w<float>(c.d.wpk);
        const bool wino = wino_geometry(c.p.B, OH, OW, cin, cout, nullptr) ||
                          (wino_span_ok() && wino_span_geometry(c.p.B, OH, OW, cin, cout, nullptr));
        if (wino) RC(launch_wino_pack(wgt, wp, cout, cin, 0, c.s));
        else RC(launch_pack_fwd(wgt, wp, cout, cin, c.s));
        ConvArgs a{};
        a.B = c.p.B; a.H = OH; a.W = OW; a.cin = cin; a.cout = cout;
        a.src = x;
        a.src_guard = 1;  // workspace tensor
        a.srcH = IH; a.srcW = IW;
        a.queue = c.p.wq ? c.w<int>(c.p.wq) : nullptr;
        a.wpack = wp;
        a.out = y;
        a.nblk = wino ? (int)wino_nblk(c.p.B, OH, OW, cin, cout) : (int)conv3x3_nblk(c.p.B, OH, OW, cout);
        a.part0 = part;
        a.part1 = part + (size_t)cout * a.nblk;
        a.partn = part + (size_t)2 * cout * a.nblk;
        {
            Scope sc(&c.p.prof, c.s, label, layer);
            RC(wino ? launch_conv3x3_wino(PRO_RAW, EPI_FWD, a, c.s) : launch_conv3x3_dma(PRO_RAW, EPI_FWD, a, c.s));
        }
        ns = a.nblk;
        f.part0 = a.part0;
        f.part1 = a.part1;
        f.partn = a.partn;
    } else {
        ConvGArgs a{};
        a.mode = 0;
        a.B = c.p.B; a.cin = cin; a.cout = cout;
        a.IH = IH; a.IW = IW; a.OH = OH; a.OW = OW;
        a.KH = a.KW = k; a.stride = stride; a.pad = pad;
        a.x = x; a.w = wgt; a.out = y;
        a.bf16 = c.d.bf16;
        a.wpack = c.w<void>(c.d.wpk16);
        a.xn = xn;
        if (train && a.bf16 && xn) {  // the channel-last engine writes the BN partials in its epilogue
            ns = (int)convn_stat_tiles(a);
            a.st_part0 = part;
            a.st_part1 = part + (size_t)cout * ns;
            a.st_partn = part + (size_t)2 * cout * ns;
            f.part0 = a.st_part0;
            f.part1 = a.st_part1;
            f.partn = a.st_partn;
        }
        Scope sc(&c.p.prof, c.s, label, layer);
        RC(launch_convg(a, c.s));
    }
    if (train && !dma_nblk && !(c.d.bf16 && xn)) {
        Scope sc(&c.p.prof, c.s, "chan_stats", strcmp(label, "shortcut_fwd") == 0 ? 100 + layer : layer);
        int bps;
        const int nsl = chan_slices(c.p.B, cout, &bps);
        f.part0 = part;
        f.part1 = part + (size_t)cout * nsl;
        f.partn = part + (size_t)2 * cout * nsl;
        RC(launch_chan_stats(y, c.p.B, cout, (int64_t)OH * OW, const_cast<float*>(f.part0),
                             const_cast<float*>(f.part1), const_cast<float*>(f.partn), &ns, c.s));
    }
    f.nblk = ns;
    f.gamma = gamma; f.beta = beta; f.bias = bias;
    f.rmean = rmean; f.rvar = rvar; f.nbt = nbt;
    f.momentum = 0.1f; f.eps = 1e-5f; f.train = train;
    f.cf = cf;
    Scope sc(&c.p.prof, c.s, "bn_fwd_finalize");
    return launch_bn_fwd_finalize(f, c.s);
}

// weight gradient of a conv into G (partials summed deterministically) + zero bias gradient
int conv_wgrad(const Ctx& c, int layer, const float* x, int cin, int IH, int IW, int k, int stride, int pad,
               const float* dy, int cout, int OH, int OW, float* gw, float* gb, const WgradArgs* w32 = nullptr,
               const float* bn_g = nullptr, const float* bn_y = nullptr, const float4* bn_cf = nullptr,
               const void* xn = nullptr, const void* dyn = nullptr, const WinoWgradArgs* ww = nullptr) {
    PCX_CHECK_ARG(x || (xn && dyn), "deep plan: weight gradient of layer %d has no input (plane or NHWC image)", layer);
    if (ww) {  // stride-1 3x3, even width: Winograd weight gradient, BN backward in its staging (dy written)
        WinoWgradArgs w = *ww;
        w.B = c.p.B; w.H = OH; w.W = OW; w.cin = cin; w.cout = cout;
        w.dz = bn_g;
        w.y = bn_y;
        w.cf_dy = bn_cf;
        w.dy_out = const_cast<float*>(dy);
        w.src = x;
        w.cf_x = nullptr;
        float* wgp = c.w<float>(c.d.wgp);
        w.part = wgp;
        { Scope sc(&c.p.prof, c.s, "wgrad", layer); RC(launch_wgrad_wino(PRO_RAW, w, c.s)); }
        RC(launch_wgrad_wino_reduce(wgp, w.nslice, cout, cin, gw, c.s));
        return hip_status_ok(hipMemsetAsync(gb, 0, (size_t)cout * 4, c.s), "memset bias grad");
    }
    if (w32) {  // stride-1 3x3: pixel-stream (wgrad_s.hip, MT 16) or 32x32 row-window (wgrad_w32.hip) kernel
        WgradArgs w = *w32;
        w.B = c.p.B; w.H = OH; w.W = OW; w.cin = cin; w.cout = cout;
        if (bn_g) {  // BN backward in the staging: dy = f(g, y) computed per row and written to `dy`
            w.dz = bn_g;
            w.y = bn_y;
            w.cf_dy = bn_cf;
            w.dy_out = const_cast<float*>(dy);
        } else {     // a ready dy (identity BN-backward coefficients)
            w.dz = dy;
            w.y = dy;
            w.cf_dy = c.w<float4>(c.d.identw);
            w.dy_out = nullptr;
        }
        w.src = x;
        w.cf_x = nullptr;
        w.drop = nullptr;
        w.srcH = IH; w.srcW = IW;
        float* wgp = c.w<float>(c.d.wgp);
        w.part = wgp;
        { Scope sc(&c.p.prof, c.s, "wgrad", layer); RC(w.MT == 16 ? launch_wgrad_s(PRO_RAW, w, c.s) : launch_wgrad_w32(PRO_RAW, w, c.s)); }
        RC(launch_sum_slices(wgp, w.nslice, (int64_t)cout * cin * 9, gw, c.s));
        return hip_status_ok(hipMemsetAsync(gb, 0, (size_t)cout * 4, c.s), "memset bias grad");
    }
    ConvGArgs a{};
    a.mode = 2;
    a.B = c.p.B; a.cin = cin; a.cout = cout;
    a.IH = IH; a.IW = IW; a.OH = OH; a.OW = OW;
    a.KH = a.KW = k; a.stride = stride; a.pad = pad;
    a.x = x; a.dy = dy;
    if (!dy) {  // BN backward of (bn_g, bn_y) applied while staging
        a.bn_g = bn_g;
        a.bn_y = bn_y;
        a.bn_cf = bn_cf;
    }
    a.bf16 = c.d.bf16;
    a.xn = xn;    // channel-last images (both set: convn.hip)
    a.dyn = dyn;
    a.nslice = convg_nslice(a, &a.kslice);
    float* wgp = c.w<float>(c.d.wgp);
    a.out = wgp;
    { Scope sc(&c.p.prof, c.s, "wgrad", layer); RC(launch_convg(a, c.s)); }
    RC(launch_sum_slices(wgp, a.nslice, (int64_t)cout * cin * k * k, gw, c.s));
    // the conv feeds a train-mode BN: d(loss)/d(bias) = sum of the BN backward = 0 exactly
    return hip_status_ok(hipMemsetAsync(gb, 0, (size_t)cout * 4, c.s), "memset bias grad");
}

int conv_dgrad(const Ctx& c, int layer, const float* dy, int cout, int OH, int OW, int k, int stride, int pad,
               const float* wgt, float* dx, int cin, int IH, int IW, int accumulate, bool dma = false,
               const void* dyn = nullptr, float* par_out = nullptr, const ConvGArgs* ep = nullptr) {
    if (dma) {  // stride-1 3x3: the LDS-DMA conv on flipped weights, plain store / accumulate
        float* wp = c.w<float>(c.d.wpk);
        const bool wino = wino_geometry(c.p.B, IH, IW, cout, cin, nullptr) ||
                          (wino_span_ok() && wino_span_geometry(c.p.B, IH, IW, cout, cin, nullptr));
        if (wino) RC(launch_wino_pack(wgt, wp, cin, cout, 1, c.s));
        else RC(launch_pack_dgrad(wgt, wp, cout, cin, c.s));
        ConvArgs a{};
        a.B = c.p.B; a.H = IH; a.W = IW; a.cin = cout; a.cout = cin;
        a.src = dy;
        a.src_guard = 1;  // workspace tensor
        a.srcH = OH; a.srcW = OW;
        a.queue = c.p.wq ? c.w<int>(c.p.wq) : nullptr;
        a.wpack = wp;
        a.out = dx;
        a.accumulate = accumulate;
        a.nblk = wino ? (int)wino_nblk(c.p.B, IH, IW, cout, cin) : (int)conv3x3_nblk(c.p.B, IH, IW, cin);
        a.part0 = a.part1 = c.w<float>(c.d.stat);
        Scope sc(&c.p.prof, c.s, "conv_dgrad", layer);
        return wino ? launch_conv3x3_wino(PRO_RAW, EPI_BWD_STORE, a, c.s) : launch_conv3x3_dma(PRO_RAW, EPI_BWD_STORE, a, c.s);
    }
    ConvGArgs a{};
    a.mode = 1;
    a.B = c.p.B; a.cin = cin; a.cout = cout;
    a.IH = IH; a.IW = IW; a.OH = OH; a.OW = OW;
    a.KH = a.KW = k; a.stride = stride; a.pad = pad;
    a.w = wgt; a.dy = dy; a.out = dx; a.accumulate = accumulate;
    a.bf16 = c.d.bf16;
    a.wpack = c.w<void>(c.d.wpk16);
    a.dyn = dyn;
    a.par_out = par_out;
    if (ep) {  // the producer BN's backward sums in the channel-last engine's epilogue
        a.ep_y = ep->ep_y; a.ep_cf = ep->ep_cf; a.ep_drop = ep->ep_drop; a.ep_pg = ep->ep_pg; a.ep_px = ep->ep_px;
    }
    Scope sc(&c.p.prof, c.s, "conv_dgrad", layer);
    return launch_convg(a, c.s);
}

// BN backward: finalize (dgamma, dbeta, coefficients) from bwd_prep partials
int bn_bwd(const Ctx& c, int C, int ns, const float* pg, const float* px, const float* gamma, const float4* cf_fwd,
           float* dgamma, float* dbeta, float4* cfb, double count) {
    BnBwdArgs f{};
    f.C = C; f.nblk = ns; f.count = count;
    f.part0 = pg; f.part1 = px;
    f.gamma = gamma; f.cf_fwd = cf_fwd;
    f.dgamma = dgamma; f.dbeta = dbeta; f.cf = cfb;
    Scope sc(&c.p.prof, c.s, "bn_bwd_finalize");
    return launch_bn_bwd_finalize(f, c.s);
}

}  // namespace

int deep_forward(const Plan& p, const float* const* P, float* const* bnstat, int64_t* const* nbt, const float* x,
                 const float* const* drop, int train, float* emb, void* ws, hipStream_t s) {
    const DeepPlan& d = *p.deep;
    const Ctx c{p, d, ws, s};
    if (p.wq) RC(hip_status_ok(hipMemsetAsync(c.w<int>(p.wq), 0, WINO_QUEUE_INTS * 4, s), "memset queue"));
    const int B = p.B;
    const float* dmask[4] = {nullptr, nullptr, nullptr, nullptr};
    if (train && drop)
        for (int i = 0; i < 4; ++i) dmask[i] = drop[i];
    auto bnp = [&](int idx, int j) { return bnstat[2 * idx + j]; };
    auto nb = [&](int idx) { return nbt ? nbt[idx] : nullptr; };
    const int C0 = d.h[0];
    // stem: direct 7x7 kernel with the BN partials in the same pass, then the BN finaliser
    {
        StemArgs sa{};
        sa.B = B; sa.H = d.H0; sa.W = d.W0; sa.cout = C0;
        sa.x = x; sa.w = P[0]; sa.out = d.stem_fused ? nullptr : c.w<float>(d.y0);  // fused: statistics only
        sa.nblk = d.stem_nblk; sa.rows_per_blk = d.stem_rows;
        float* part = c.w<float>(d.stat);
        sa.part0 = part;
        sa.part1 = part + (size_t)C0 * sa.nblk;
        sa.partn = part + (size_t)2 * C0 * sa.nblk;
        { Scope sc(&p.prof, s, "conv_fwd", 0); RC(launch_stem_fwd(sa, d.bf16, c.w<float>(d.stemw), s)); }
        BnFwdArgs f{};
        f.C = C0; f.nblk = sa.nblk;
        f.part0 = sa.part0; f.part1 = sa.part1; f.partn = sa.partn;
        f.gamma = P[2]; f.beta = P[3]; f.bias = P[1];
        f.rmean = bnp(0, 0); f.rvar = bnp(0, 1); f.nbt = nb(0);
        f.momentum = 0.1f; f.eps = 1e-5f; f.train = train;
        f.cf = c.w<float4>(d.cf0);
        Scope sc(&p.prof, s, "bn_fwd_finalize");
        RC(launch_bn_fwd_finalize(f, s));
    }
    if (d.stem_fused) {  // y0 recomputed: a0, taps, y0 at the taps and block 0's NHWC input in one pass
        StemArgs sa{};
        sa.B = B; sa.H = d.H0; sa.W = d.W0; sa.cout = C0;
        sa.x = x; sa.w = c.w<float>(d.stemw);
        sa.cf = c.w<float4>(d.cf0);
        sa.pool_arg = c.w<uint8_t>(d.mparg); sa.pool_ysel = c.w<float>(d.ysel);  // pooled NHWC; no a0 plane
        sa.pool_nhwc = d.blk[0].cn ? c.w<void>(d.blk[0].an) : nullptr;
        sa.OH = d.H1; sa.OW = d.W1;
        Scope sc(&p.prof, s, "maxpool_fwd");
        RC(launch_stem_pool(sa, s));
    } else {
        Scope sc(&p.prof, s, "maxpool_fwd");
        RC(launch_maxpool3_fwd(c.w<float>(d.y0), c.w<float4>(d.cf0), c.w<float>(d.a0), c.w<uint8_t>(d.mparg), B, C0,
                               d.H0, d.W0, d.H1, d.W1, s));
    }
    const float* a = c.w<float>(d.a0);
    for (int i = 0; i < 4; ++i) {
        const DeepBlock& k = d.blk[i];
        const int q = k.pidx, L = 2 * i + 1;
        const void* an = k.cn ? c.w<void>(k.an) : nullptr;
        const void* d1n = k.cn ? c.w<void>(k.d1n) : nullptr;
        // (otherwise written by the previous block's activation -- whenever this block is channel-last,
        // whatever the previous block's engine -- or for block 0 by the fused stem pool)
        if (k.cn && i == 0 && !d.stem_fused) {
            Scope sc(&p.prof, s, "to_nhwc", L);
            RC(launch_to_nhwc(nhwc_args(NHWC_COPY, B, k.cin, k.Hi, k.Wi, a, c.w<void>(k.an)), s));
        }
        RC(conv_bn_fwd(c, "conv_fwd", L, a, k.cin, k.Hi, k.Wi, 3, k.stride, 1, P[q], c.w<float>(k.y1), k.cout, k.Ho,
                       k.Wo, P[q + 2], P[q + 3], P[q + 1], bnp(k.bnidx, 0), bnp(k.bnidx, 1), nb(k.bnidx), train,
                       c.w<float4>(k.cf1), k.dma1 ? k.nblk1 : 0, an));
        const int64_t P2 = (int64_t)k.Ho * k.Wo;
        {
            Scope sc(&p.prof, s, "bn_act", L);
            if (k.cn) {  // d1 feeds only conv2 (forward and weight gradient): its channel-last image alone
                NhwcArgs t = nhwc_args(NHWC_ACT, B, k.cout, k.Ho, k.Wo, c.w<float>(k.y1), c.w<void>(k.d1n));
                t.cf = c.w<float4>(k.cf1);
                t.drop = d.residual ? dmask[i] : nullptr;
                RC(launch_to_nhwc(t, s));
            } else {
                RC(launch_bn_act(c.w<float>(k.y1), c.w<float4>(k.cf1), nullptr, nullptr,
                                 d.residual ? dmask[i] : nullptr, c.w<float>(k.d1), B, k.cout, P2, s));
            }
        }
        RC(conv_bn_fwd(c, "conv_fwd", L + 1, c.w<float>(k.d1), k.cout, k.Ho, k.Wo, 3, 1, 1, P[q + 4], c.w<float>(k.y2),
                       k.cout, k.Ho, k.Wo, P[q + 6], P[q + 7], P[q + 5], bnp(k.bnidx + 1, 0), bnp(k.bnidx + 1, 1),
                       nb(k.bnidx + 1), train, c.w<float4>(k.cf2), k.dma2 ? k.nblk2 : 0, d1n));
        const float* res = nullptr;
        const float4* rcf = nullptr;
        if (k.sc) {
            RC(conv_bn_fwd(c, "shortcut_fwd", i, a, k.cin, k.Hi, k.Wi, 1, k.stride, 0, P[q + 8], c.w<float>(k.ysc),
                           k.cout, k.Ho, k.Wo, P[q + 10], P[q + 11], P[q + 9], bnp(k.bnidx + 2, 0),
                           bnp(k.bnidx + 2, 1), nb(k.bnidx + 2), train, c.w<float4>(k.cfsc), 0, an));
            res = c.w<float>(k.ysc);
            rcf = c.w<float4>(k.cfsc);
        } else if (d.residual) {
            PCX_CHECK_ARG(a, "deep plan: identity residual of block %d reads a byte-masked output", i);
            res = a;
        }
        // fused stem: block 0's identity residual a0 = relu(BN0(y0 at the tap)) from the pooled NHWC y0
        const bool res_pool = i == 0 && d.stem_fused && res == a;
        if (res_pool) {
            res = c.w<float>(d.ysel);
            rcf = c.w<float4>(d.cf0);
        }
        {
            Scope sc(&p.prof, s, "bn_act", L + 1);
            if (i < 3 && d.blk[i + 1].cn) {  // the block output and the next block's channel-last input
                NhwcArgs t = nhwc_args(NHWC_ACT, B, k.cout, k.Ho, k.Wo, c.w<float>(k.y2), c.w<void>(d.blk[i + 1].an));
                t.cf = c.w<float4>(k.cf2);
                t.res = res;
                t.rcf = rcf;
                t.res_pool = res_pool ? 1 : 0;
                t.drop = d.residual ? nullptr : dmask[i];
                // the float32 output is read only as the backward's ReLU mask (residual) or not at all
                t.out32 = k.m8 ? nullptr : c.w<float>(k.out);
                t.mask8 = k.m8 ? c.w<uint8_t>(k.m8) : nullptr;
                RC(launch_to_nhwc(t, s));
            } else {
                RC(launch_bn_act(c.w<float>(k.y2), c.w<float4>(k.cf2), res, rcf, d.residual ? nullptr : dmask[i],
                                 c.w<float>(k.out), B, k.cout, P2, s));
            }
        }
        a = block_out(c, i);  // nullptr under the byte mask: the next block reads only its NHWC image
    }
    // head on the (already non-negative) trunk output: identity BN coefficients
    RC(launch_fill_cf(c.w<float4>(d.ident), d.h[3], make_float4(1.f, 0.f, 0.f, 1.f), s));
    {
        HeadPoolArgs h{};
        h.B = B; h.C = p.C6; h.P = p.P6;
        h.y = a;
        h.cf = c.w<float4>(d.ident);
        h.drop = nullptr;
        h.wa = p.cfg.use_attention ? P[d.ia] : nullptr;
        h.ba = p.cfg.use_attention ? P[d.ia + 1] : nullptr;
        h.pooled = at<float>(ws, p.pooled);
        h.att = at<float>(ws, p.att);
        Scope sc(&p.prof, s, "head_pool_fwd");
        RC(launch_head_pool_fwd(h, s));
    }
    {
        const int ip = d.ip;
        RC(launch_transpose(P[ip], at<float>(ws, p.wt), p.D, p.C6, s));
        ProjArgs j{};
        j.B = B; j.K = p.C6; j.D = p.D;
        j.pooled = at<float>(ws, p.pooled);
        j.w = P[ip];
        j.wt = at<float>(ws, p.wt);
        j.bias = P[ip + 1];
        j.gamma = P[ip + 2];
        j.beta = P[ip + 3];
        j.rmean = bnp(d.bn_proj, 0);
        j.rvar = bnp(d.bn_proj, 1);
        j.nbt = nb(d.bn_proj);
        j.momentum = 0.1f;
        j.eps = 1e-5f;
        j.train = train;
        j.h = at<float>(ws, p.h);
        j.cf = at<float4>(ws, p.cfp);
        j.emb = emb;
        j.norm = at<float>(ws, p.norm);
        Scope sc(&p.prof, s, "proj_fwd");
        RC(launch_proj_fwd(j, s));
    }
    return PCX_OK;
}

int deep_backward(const Plan& p, const float* const* P, const float* x, const float* const* drop, const float* emb,
                  const float* demb, float* const* G, void* ws, hipStream_t s) {
    const DeepPlan& d = *p.deep;
    const Ctx c{p, d, ws, s};
    if (p.wq) RC(hip_status_ok(hipMemsetAsync(c.w<int>(p.wq), 0, WINO_QUEUE_INTS * 4, s), "memset queue"));
    const int B = p.B;
    const float* dmask[4] = {nullptr, nullptr, nullptr, nullptr};
    if (drop)
        for (int i = 0; i < 4; ++i) dmask[i] = drop[i];
    float* part = c.w<float>(d.stat);
    const int ip = d.ip, ia = d.ia;
    // dy is handed to the routed weight gradients ready-made: identity BN-backward coefficients
    RC(launch_fill_cf(c.w<float4>(d.identw), d.cmax, make_float4(1.f, 0.f, 0.f, 1.f), s));
    p.buckets.begin();
    {
        ProjArgs j{};
        j.B = B; j.K = p.C6; j.D = p.D;
        j.pooled = at<float>(ws, p.pooled);
        j.w = P[ip];
        j.gamma = P[ip + 2];
        j.h = at<float>(ws, p.h);
        j.cf = at<float4>(ws, p.cfp);
        j.emb = const_cast<float*>(emb);
        j.norm = at<float>(ws, p.norm);
        j.demb = demb;
        j.dzp = at<float>(ws, p.dzp);
        j.cfb = at<float4>(ws, p.cfpb);
        j.dh = at<float>(ws, p.dh);
        j.dpooled = at<float>(ws, p.dpooled);
        j.dw = G[ip];
        j.db = G[ip + 1];
        j.dgamma = G[ip + 2];
        j.dbeta = G[ip + 3];
        j.part = at<float>(ws, p.proj_part);
        Scope sc(&p.prof, s, "proj_bwd");
        RC(launch_proj_bwd(j, s));
    }
    p.buckets.mark(ip, s);
    {
        HeadPoolArgs h{};
        h.B = B; h.C = p.C6; h.P = p.P6;
        h.y = c.w<float>(d.blk[3].out);
        h.cf = c.w<float4>(d.ident);
        h.drop = nullptr;
        h.wa = p.cfg.use_attention ? P[ia] : nullptr;
        h.ba = p.cfg.use_attention ? P[ia + 1] : nullptr;
        h.att = at<float>(ws, p.att);
        h.dpooled = at<float>(ws, p.dpooled);
        h.dz = c.w<float>(d.hdz);
        h.p_dz = part;
        h.p_dzx = part + (size_t)p.C6 * B;
        h.p_dwa = at<float>(ws, p.hp_dwa);
        h.p_dba = at<float>(ws, p.hp_dba);
        { Scope sc(&p.prof, s, "head_pool_bwd"); RC(launch_head_pool_bwd(h, s)); }
        if (p.cfg.use_attention) {
            RC(launch_row_sum(h.p_dwa, p.C6, B, G[ia], s));
            RC(launch_row_sum(h.p_dba, 1, B, G[ia + 1], s));
            p.buckets.mark(ia, s);
        }
    }
    // upstream gradient of the current block's output (already ReLU-masked for the last block)
    const float* dout = c.w<float>(d.hdz);
    const float* dout2 = nullptr;  // block 0's shortcut gradient, added by the fused stem backward
    // a stride-2 block's input gradient left in its parity-class planes (d.partmp): the previous
    // block's BN backward prep reads them directly (no interleave pass)
    const float* dpar = nullptr;
    int64_t dpo[4] = {0, 0, 0, 0};
    bool masked = true;
    for (int i = 3; i >= 0; --i) {
        const DeepBlock& k = d.blk[i];
        const int q = k.pidx, L = 2 * i + 1;
        const int64_t P2 = (int64_t)k.Ho * k.Wo;
        const double count = (double)B * P2;
        const float* a_in = i == 0 ? c.w<float>(d.a0) : block_out(c, i - 1);  // nullptr: byte-masked
        float* g = c.w<float>(d.g);
        float* dy2 = c.w<float>(d.dyA);
        float* dysc = c.w<float>(d.dyB);
        int ns = 0;
        // ---- g = dL/d(pre-activation sum) (residual) or dL/d(BN2 output) (plain); BN2 [+ BNsc] sums
        {
            BwdPrepArgs b{};
            b.B = B; b.C = k.cout; b.P = P2;
            b.d = dout;
            if (dpar) {
                b.dpar = dpar;
                for (int q2 = 0; q2 < 4; ++q2) b.dpo[q2] = dpo[q2];
                b.H = k.Ho; b.W = k.Wo;
            }
            if (d.residual) {
                b.mask_mode = masked ? MASK_NONE : (k.m8 ? MASK_OUT8 : MASK_OUT);
                b.mask_src = block_out(c, i);
                b.mask8 = k.m8 ? c.w<uint8_t>(k.m8) : nullptr;
            } else {
                b.mask_mode = MASK_BN;
                b.mask_src = c.w<float>(k.y2);
                b.mask_cf = c.w<float4>(k.cf2);
                b.drop = dmask[i];
            }
            b.g = g;
            b.y1 = c.w<float>(k.y2);
            b.cf1 = c.w<float4>(k.cf2);
            if (k.sc) { b.y2 = c.w<float>(k.ysc); b.cf2 = c.w<float4>(k.cfsc); }
            int bps;
            const int nsl = chan_slices(B, k.cout, &bps);
            b.p_g = part;
            b.p_x1 = part + (size_t)k.cout * nsl;
            b.p_x2 = k.sc ? part + (size_t)2 * k.cout * nsl : nullptr;
            { Scope sc(&p.prof, s, "bwd_prep", L + 1); RC(launch_bwd_prep(b, &ns, s)); }
            RC(bn_bwd(c, k.cout, ns, b.p_g, b.p_x1, P[q + 6], c.w<float4>(k.cf2), G[q + 6], G[q + 7],
                      c.w<float4>(k.cfb2), count));
            if (k.sc)
                RC(bn_bwd(c, k.cout, ns, b.p_g, b.p_x2, P[q + 10], c.w<float4>(k.cfsc), G[q + 10], G[q + 11],
                          c.w<float4>(k.cfbsc), count));
        }
        // channel-last bf16 dy images: the BN backward applied while converting (no float32 dy)
        const void* an = k.cn ? c.w<void>(k.an) : nullptr;
        const void* d1n = k.cn ? c.w<void>(k.d1n) : nullptr;
        void* dyn1 = k.cn ? c.w<void>(d.dyn1) : nullptr;
        void* dyn2 = k.cn ? c.w<void>(d.dyn2) : nullptr;
        if (k.cn) {
            Scope sc(&p.prof, s, "dy_nhwc", L + 1);
            NhwcArgs t = nhwc_args(NHWC_BNBWD, B, k.cout, k.Ho, k.Wo, g, dyn1);
            t.y = c.w<float>(k.y2);
            t.cf = c.w<float4>(k.cfb2);
            if (k.sc) {  // the shortcut's dy image from the same g in the same pass
                t.y_b = c.w<float>(k.ysc);
                t.cf_b = c.w<float4>(k.cfbsc);
                t.dst_b = dyn2;
            }
            RC(launch_to_nhwc(t, s));
        } else {
            Scope sc(&p.prof, s, "bn_bwd_apply", L + 1);
            // (a routed conv2's dy is produced by its weight-gradient kernel's staging)
            if (!k.w32_2) RC(launch_bn_bwd_apply(g, c.w<float>(k.y2), c.w<float4>(k.cfb2), dy2, B, k.cout, P2, s));
            if (k.sc) RC(launch_bn_bwd_apply(g, c.w<float>(k.ysc), c.w<float4>(k.cfbsc), dysc, B, k.cout, P2, s));
        }
        // ---- conv2
        RC(conv_wgrad(c, L + 1, c.w<float>(k.d1), k.cout, k.Ho, k.Wo, 3, 1, 1, dy2, k.cout, k.Ho, k.Wo, G[q + 4],
                      G[q + 5], k.w32_2 ? &k.wg2 : nullptr, g, c.w<float>(k.y2), c.w<float4>(k.cfb2), d1n, dyn1,
                      k.ww2 ? &k.wwa2 : nullptr));
        float* dd = c.w<float>(d.dd);
        // channel-last: conv2's data gradient also reduces BN1's backward sums (no bwd_prep pass over dd)
        const bool ep_sums = k.cn && !PCX_AB_NO_EPSUMS;
        ConvGArgs ep{};
        if (ep_sums) {
            ConvGArgs q{};  // conv2's data gradient: its epilogue tiles
            q.mode = 1; q.B = B; q.IH = q.OH = k.Ho; q.IW = q.OW = k.Wo; q.KH = q.KW = 3; q.stride = 1; q.pad = 1;
            ns = (int)convn_stat_tiles(q);
            ep.ep_y = c.w<float>(k.y1);
            ep.ep_cf = c.w<float4>(k.cf1);
            ep.ep_drop = d.residual ? dmask[i] : nullptr;
            ep.ep_pg = part;
            ep.ep_px = part + (size_t)k.cout * ns;
        }
        RC(conv_dgrad(c, L + 1, dy2, k.cout, k.Ho, k.Wo, 3, 1, 1, P[q + 4], dd, k.cout, k.Ho, k.Wo, 0, k.dma2, dyn1,
                      nullptr, ep_sums ? &ep : nullptr));
        // ---- through Dropout2d / ReLU / BN1
        if (ep_sums) {
            RC(bn_bwd(c, k.cout, ns, ep.ep_pg, ep.ep_px, P[q + 2], c.w<float4>(k.cf1), G[q + 2], G[q + 3],
                      c.w<float4>(k.cfb1), count));
        } else {
            BwdPrepArgs b{};
            b.B = B; b.C = k.cout; b.P = P2;
            b.d = dd;
            b.mask_mode = MASK_BN;
            b.mask_src = c.w<float>(k.y1);
            b.mask_cf = c.w<float4>(k.cf1);
            b.drop = d.residual ? dmask[i] : nullptr;
            b.g = k.cn ? nullptr : dd;  // channel-last: the dy writer re-applies the mask to dd itself
            b.y1 = c.w<float>(k.y1);
            b.cf1 = c.w<float4>(k.cf1);
            int bps;
            const int nsl = chan_slices(B, k.cout, &bps);
            b.p_g = part;
            b.p_x1 = part + (size_t)k.cout * nsl;
            { Scope sc(&p.prof, s, "bwd_prep", L); RC(launch_bwd_prep(b, &ns, s)); }
            RC(bn_bwd(c, k.cout, ns, b.p_g, b.p_x1, P[q + 2], c.w<float4>(k.cf1), G[q + 2], G[q + 3],
                      c.w<float4>(k.cfb1), count));
        }
        float* dy1 = dy2;  // dy2 (and its image) are dead after conv2's gradients
        if (k.cn) {
            Scope sc(&p.prof, s, "dy_nhwc", L);
            NhwcArgs t = nhwc_args(NHWC_BNBWD, B, k.cout, k.Ho, k.Wo, dd, dyn1);
            t.y = c.w<float>(k.y1);
            t.cf = c.w<float4>(k.cfb1);
            t.mcf = c.w<float4>(k.cf1);
            t.drop = d.residual ? dmask[i] : nullptr;
            RC(launch_to_nhwc(t, s));
        } else {
            Scope sc(&p.prof, s, "bn_bwd_apply", L);
            if (!k.w32_1) RC(launch_bn_bwd_apply(dd, c.w<float>(k.y1), c.w<float4>(k.cfb1), dy1, B, k.cout, P2, s));
        }
        // ---- conv1 (+ shortcut): gradients of the weights and of the block input
        RC(conv_wgrad(c, L, a_in, k.cin, k.Hi, k.Wi, 3, k.stride, 1, dy1, k.cout, k.Ho, k.Wo, G[q], G[q + 1],
                      k.w32_1 ? &k.wg1 : nullptr, dd, c.w<float>(k.y1), c.w<float4>(k.cfb1), an, dyn1,
                      k.ww1 ? &k.wwa1 : nullptr));
        float* da = c.w<float>(k.da);
        int acc = 0;
        // identity shortcut: the block input receives g directly -- for block 0 of the fused stem the
        // stem's pooled backward adds it while loading (no copy, no accumulating data gradient)
        const bool sc_in_stem = i == 0 && d.residual && !k.sc &&
                                (d.stem_fused || maxpool3_bwd_prep_fits(d.H0, d.W0, d.H1, d.W1));
        if (d.residual && !k.sc && !sc_in_stem) {
            RC(hip_status_ok(hipMemcpyAsync(da, g, (size_t)B * k.cout * P2 * 4, hipMemcpyDeviceToDevice, s),
                             "copy shortcut grad"));
            acc = 1;
        }
        // stride 2 (fp32 / channel-last engines): the parity classes go dense into class planes (the
        // shortcut's class accumulates there too), then one pass interleaves them into da
        float* ptmp = k.planar ? c.w<float>(d.partmp) : nullptr;
        RC(conv_dgrad(c, L, dy1, k.cout, k.Ho, k.Wo, 3, k.stride, 1, P[q], da, k.cin, k.Hi, k.Wi, k.planar ? 0 : acc,
                      k.dma1, dyn1, ptmp));
        if (k.sc) {
            RC(conv_wgrad(c, 100 + i, a_in, k.cin, k.Hi, k.Wi, 1, k.stride, 0, dysc, k.cout, k.Ho, k.Wo, G[q + 8],
                          G[q + 9], nullptr, nullptr, nullptr, nullptr, an, dyn2));
            RC(conv_dgrad(c, 100 + i, dysc, k.cout, k.Ho, k.Wo, 1, k.stride, 0, P[q + 8], da, k.cin, k.Hi, k.Wi, 1,
                          false, dyn2, ptmp));
        }
        dpar = nullptr;
        if (k.planar) {
            if (i > 0 && !acc) {  // consumed only by block i - 1's BN backward prep: read in place
                dpar = ptmp;
                for (int q2 = 0; q2 < 4; ++q2) dpo[q2] = par_off(B, k.cin, k.Hi, k.Wi, q2);
            } else {
                Scope sc(&p.prof, s, "dgrad_interleave", L);
                RC(launch_par_interleave(ptmp, da, B, k.cin, k.Hi, k.Wi, acc, s));
            }
        }
        dout = dpar ? nullptr : da;
        dout2 = sc_in_stem ? g : nullptr;
        masked = false;
        p.buckets.mark(k.pidx, s);
    }
    // ---- stem: MaxPool(3,2,1) + ReLU backward, BN0 backward, 7x7 weight gradient
    const int C0 = d.h[0];
    const int64_t P0 = (int64_t)d.H0 * d.W0;
    float* dz0 = c.w<float>(d.dz0);
    if (d.stem_fused) {  // dz0 as bf16 + BN0 sums over the windows (stem_pool_bwd_kernel)
        StemArgs sa{};
        sa.B = B; sa.H = d.H0; sa.W = d.W0; sa.cout = C0; sa.OH = d.H1; sa.OW = d.W1;
        sa.cf = c.w<float4>(d.cf0);
        sa.pool_arg = c.w<uint8_t>(d.mparg);
        sa.pool_ysel = c.w<float>(d.ysel);
        sa.dpool = dout;
        sa.dpool2 = dout2;
        sa.dz16 = c.w<uint16_t>(d.dz0);
        sa.p_g = part;
        sa.p_x = part + (size_t)C0 * B;  // partials [C0][B]
        int ns;
        {
            Scope sc(&p.prof, s, "maxpool_bwd");
            RC(launch_stem_pool_bwd(sa, &ns, s));
        }
        RC(bn_bwd(c, C0, ns, sa.p_g, sa.p_x, P[2], c.w<float4>(d.cf0), G[2], G[3], c.w<float4>(d.cfb0), (double)B * P0));
    } else if (maxpool3_bwd_prep_fits(d.H0, d.W0, d.H1, d.W1)) {  // one pass: pooled gradient + BN0 sums
        int bps, ns;
        const int nsl = chan_slices(B, C0, &bps);
        float* p_g = part;
        float* p_x = part + (size_t)C0 * nsl;
        {
            Scope sc(&p.prof, s, "maxpool_bwd");
            RC(launch_maxpool3_bwd_prep(c.w<uint8_t>(d.mparg), dout, c.w<float>(d.y0), nullptr, c.w<float4>(d.cf0), dz0,
                                        p_g, p_x, B, C0, d.H0, d.W0, d.H1, d.W1, &ns, s, dout2));
        }
        RC(bn_bwd(c, C0, ns, p_g, p_x, P[2], c.w<float4>(d.cf0), G[2], G[3], c.w<float4>(d.cfb0), (double)B * P0));
    } else {
        {
            Scope sc(&p.prof, s, "maxpool_bwd");
            RC(launch_maxpool3_bwd(c.w<uint8_t>(d.mparg), dout, dz0, B, C0, d.H0, d.W0, d.H1, d.W1, s));
        }
        BwdPrepArgs b{};
        b.B = B; b.C = C0; b.P = P0;
        b.d = dz0;
        b.mask_mode = MASK_NONE;
        b.g = dz0;
        b.y1 = c.w<float>(d.y0);
        b.cf1 = c.w<float4>(d.cf0);
        int bps, ns;
        const int nsl = chan_slices(B, C0, &bps);
        b.p_g = part;
        b.p_x1 = part + (size_t)C0 * nsl;
        { Scope sc(&p.prof, s, "bwd_prep", 0); RC(launch_bwd_prep(b, &ns, s)); }
        RC(bn_bwd(c, C0, ns, b.p_g, b.p_x1, P[2], c.w<float4>(d.cf0), G[2], G[3], c.w<float4>(d.cfb0),
                  (double)B * P0));
    }
    // the stem's dy feeds only its weight gradient: the direct stem kernel applies the BN backward
    // to (dz0, y0) as it loads them (no dy pass)
    {
        StemArgs sa{};
        sa.B = B; sa.H = d.H0; sa.W = d.W0; sa.cout = C0;
        sa.x = x; sa.dz = dz0; sa.dz16 = c.w<uint16_t>(d.dz0); sa.cf_dy = c.w<float4>(d.cfb0);
        float* wgp = c.w<float>(d.wgp);
        sa.part = wgp;
        sa.nblk = d.stem_ns; sa.rows_per_blk = d.stem_srows;
        if (d.stem_fused) {  // y0 recomputed from the bf16-rounded weights of the forward
            sa.w = c.w<float>(d.stemw);
            Scope sc(&p.prof, s, "wgrad", 0);
            RC(launch_stem_wgrad_rc(sa, s));
        } else {
            sa.y = c.w<float>(d.y0);
            Scope sc(&p.prof, s, "wgrad", 0);
            RC(launch_stem_wgrad(sa, d.bf16, s));
        }
        RC(launch_sum_slices(wgp, sa.nblk, (int64_t)C0 * 49, G[0], s));
        // the stem conv feeds a train-mode BN: its bias gradient is exactly 0
        RC(hip_status_ok(hipMemsetAsync(G[1], 0, (size_t)C0 * 4, s), "memset bias grad"));
    }
    p.buckets.mark(0, s);
    return PCX_OK;
}

}  // namespace pcx
