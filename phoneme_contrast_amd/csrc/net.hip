// Network plans: the whole PhonemeNet forward / backward as one C-ABI call each.
//
// A plan is an immutable host object (shapes, launch geometry, workspace carve-out).  The caller
// owns every device buffer: parameters and gradients (reference state_dict order), BN running
// statistics, dropout masks and one workspace of pcx_net_workspace_bytes().  The forward leaves
// the raw conv outputs y1..y6 and the head state in the workspace; the backward consumes them.
//
// cnn_small (reference src/models/phoneme_cnn.py:10-126):
//   y1 = conv1(x)                         z = BN(y), r = ReLU(z)     (BN/ReLU never stored)
//   y2 = conv2(r1)          x3 = Dropout2d(MaxPool2(r2))   y3 = conv3(x3)
//   y4 = conv4(r3)          x5 = Dropout2d(MaxPool2(r4))   y5 = conv5(x5)
//   y6 = conv6(r5)          x6 = Dropout2d(r6) -> attention -> mean -> Linear -> BN1d -> normalize
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "plan.h"

namespace pcx {

// parameter indices (state_dict / named_parameters order) for cnn_small
static inline int p_conv_w(int L) { return 8 * ((L - 1) / 2) + 4 * ((L - 1) % 2); }
static inline int p_conv_b(int L) { return p_conv_w(L) + 1; }
static inline int p_bn_g(int L) { return p_conv_w(L) + 2; }
static inline int p_bn_b(int L) { return p_conv_w(L) + 3; }

int build_small(Plan& p) {
    const int B = p.B, H1 = p.F, W1 = p.T;
    PCX_CHECK_ARG(H1 >= 4 && W1 >= 4, "PhonemeNet needs n_mfcc >= 4 and T >= 4 (got %d x %d)", H1, W1);
    const int H3 = H1 / 2, W3 = W1 / 2, H5 = H3 / 2, W5 = W3 / 2;
    struct { int cin, cout, H, W, srcH, srcW, pooled, drop; } spec[7] = {
        {0, 0, 0, 0, 0, 0, 0, -1},
        {1, 32, H1, W1, H1, W1, 0, -1},
        {32, 32, H1, W1, H1, W1, 0, -1},
        {32, 64, H3, W3, H1, W1, 1, 0},
        {64, 64, H3, W3, H3, W3, 0, -1},
        {64, 128, H5, W5, H3, W3, 1, 1},
        {128, 128, H5, W5, H5, W5, 0, -1},
    };
    size_t stat = 0, wg = 0;
    for (int l = 1; l <= 6; ++l) {
        Layer& L = p.L[l];
        L.cin = spec[l].cin; L.cout = spec[l].cout; L.H = spec[l].H; L.W = spec[l].W;
        L.srcH = spec[l].srcH; L.srcW = spec[l].srcW; L.pooled_in = spec[l].pooled; L.drop_idx = spec[l].drop;
        size_t n = (size_t)B * L.cout * L.H * L.W;
        char nm[16];
        snprintf(nm, sizeof nm, "y%d", l);
        L.y = p.carve(nm, n * 4);
        snprintf(nm, sizeof nm, "dz%d", l);
        L.dz = p.carve(nm, n * 4);
        snprintf(nm, sizeof nm, "cf%d", l);
        L.cf = p.carve(nm, L.cout * 16);
        snprintf(nm, sizeof nm, "cfb%d", l);
        L.cfb = p.carve(nm, L.cout * 16);
        if (L.pooled_in) {
            snprintf(nm, sizeof nm, "xp%d", l);
            L.xp = p.carve(nm, (size_t)B * L.cin * L.H * L.W * 4);
        }
        if (l >= 2) {
            L.wino = wino_geometry(B, L.H, L.W, L.cin, L.cout, nullptr) &&
                     wino_geometry(B, L.H, L.W, L.cout, L.cin, nullptr);
            L.wu = p.carve("wu", (size_t)16 * L.cin * L.cout * 4);
            L.wud = p.carve("wud", (size_t)16 * L.cin * L.cout * 4);
            // the data gradient's tile blocks are the forward's (same H x W), so one nblk serves both
            if (L.pooled_in && L.wino && !PCX_AB_NO_POOLSEL) {
                snprintf(nm, sizeof nm, "ysel%d", l);
                L.ysel = p.carve(nm, (size_t)B * L.cin * L.H * L.W * 4);
                snprintf(nm, sizeof nm, "parg%d", l);
                L.parg = p.carve(nm, (size_t)B * L.cin * L.H * L.W);
            }
            L.nblk = L.wino ? (int)wino_nblk(B, L.H, L.W, L.cin, L.cout)
                            : (int)std::max(conv3x3_nblk(B, L.H, L.W, L.cout), conv3x3_nblk(B, L.H, L.W, L.cin));
            L.wgw = wgrad_wino_geometry(B, L.H, L.W, L.cin, L.cout, &L.ww);
            // layer 2 (32 -> 32 at full resolution, BN + ReLU input): both gradients in one pass
            L.wgbd = l == 2 && !L.pooled_in && L.cin == 32 && L.cout == 32 && L.wino && !PCX_AB_NO_WGBD &&
                     wgbd_wino_geometry(B, L.H, L.W, 32, &L.wb);
            if (L.wgbd) {
                wg = std::max(wg, (size_t)L.wb.nslice * 32 * 32 * 16);
                stat = std::max(stat, (size_t)2 * 32 * L.wb.nslice);
            }
            if (L.wgw) {
                wg = std::max(wg, (size_t)L.ww.nslice * L.cout * L.cin * 16);
            } else {
                PCX_CHECK_ARG(wgrad_s_geometry(B, L.H, L.W, L.cin, L.cout, &L.wg),
                              "PhonemeNet: no weight-gradient geometry for layer %d (%dx%d)", l, L.H, L.W);
                wg = std::max(wg, (size_t)L.wg.nslice * L.cout * L.cin * 9);
            }
        } else {
            L.nblk = conv1_nblk(B, L.H, &p.conv1_rows);
            p.conv1_nblk = L.nblk;
        }
        stat = std::max(stat, (size_t)2 * L.cout * L.nblk + L.nblk);
    }
    {  // layer 2's fused backward reads layer 3's pooled data gradient + selection (a quarter of dz2's bytes)
        Layer &L2 = p.L[2], &L3 = p.L[3];
        L2.pd = L2.wgbd && L3.pooled_in && L3.ysel && L3.wino && !(L2.H & 1) && L2.W % 4 == 0 &&
                L3.H == L2.H / 2 && L3.W == L2.W / 2 && !PCX_AB_NO_POOLDZ;
        for (int i = 0; L2.pd && i < L2.wb.nseg; ++i) L2.pd = !(L2.wb.seg_t0[i] & 1);
        // likewise layer 4's Winograd weight gradient behind layer 5's pool (its data gradient reads dy)
        Layer &L4 = p.L[4], &L5 = p.L[5];
        L4.pd = L4.wgw && !L4.wgbd && !L4.pooled_in && L5.pooled_in && L5.ysel && L5.wino && !(L4.H & 1) &&
                L4.W % 4 == 0 && L4.ww.V == 4 && (L4.ww.nseg == 1 || !(L4.ww.S & 1)) && L5.H == L4.H / 2 &&
                L5.W == L4.W / 2 && !PCX_AB_NO_POOLDZ;
    }
    // (round 6) the block tails behind layers 2 / 4: the producer's forward epilogue makes the 2x2 pool selection
    // (its tiles are the windows), so the pooled activation is a light pass over the selected values
    for (int l = 3; l <= 5; l += 2) {
        Layer &L = p.L[l], &Lp = p.L[l - 1];
        L.psel = L.pooled_in && L.ysel && Lp.wino && Lp.cin % 8 == 0 && !(Lp.H & 1) && !(Lp.W & 1) &&
                 L.H == Lp.H / 2 && L.W == Lp.W / 2 && (L.H * L.W) % 4 == 0 && !PCX_AB_NO_PSEL;
    }
    // first-layer weight gradient slices
    {
        p.wg1_nslice = wgrad1_nslice(B, H1, W1, 32, &p.wg1_rows);
        wg = std::max(wg, (size_t)p.wg1_nslice * 32 * 9);
    }
    p.C6 = 128;
    p.P6 = H5 * W5;
    stat = std::max(stat, (size_t)2 * p.C6 * B);
    p.stat_part = p.carve("stat_part", stat * 4);
    // the Winograd convs take their units from a per-XCD queue (PCX_AB_NO_WINO_QUEUE: static order)
    p.wq = PCX_AB_NO_WINO_QUEUE ? 0 : p.carve("wino_queue", WINO_QUEUE_INTS * 4);
    {
        size_t dymax = 0;
        for (int l = 2; l <= 6; ++l) dymax = std::max(dymax, (size_t)B * p.L[l].cout * p.L[l].H * p.L[l].W);
        p.dyb = p.carve("dy", dymax * 4);
    }
    p.wg_part = p.carve("wg_part", wg * 4);
    const int D = p.D, K = p.C6;
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
    p.hp_dz = p.carve("hp_dz", (size_t)K * B * 4);
    p.hp_dzx = p.carve("hp_dzx", (size_t)K * B * 4);
    p.hp_dwa = p.carve("hp_dwa", (size_t)K * B * 4);
    p.hp_dba = p.carve("hp_dba", (size_t)B * 4);
    p.nparams = p.cfg.use_attention ? 30 : 28;
    // backward completion points: projection, attention, then conv layers 6..1
    p.stages = {p.cfg.use_attention ? 26 : 24};
    if (p.cfg.use_attention) p.stages.push_back(24);
    for (int l = 6; l >= 1; --l) p.stages.push_back(p_conv_w(l));
    p.nbn = 7;
    p.ndrop = 3;
    p.drop_ch[0] = 32; p.drop_ch[1] = 64; p.drop_ch[2] = 128;
    return PCX_OK;
}


int small_forward(const Plan& p, const float* const* P, float* const* bnstat, int64_t* const* nbt,
                  const float* x, const float* const* drop, int train, float* emb, void* ws,
                  hipStream_t s) {
    const int B = p.B;
    if (p.wq) RC(hip_status_ok(hipMemsetAsync(at<int>(ws, p.wq), 0, WINO_QUEUE_INTS * 4, s), "memset queue"));
    const float mom = 0.1f, eps = 1e-5f;
    const float* dmask[3] = {nullptr, nullptr, nullptr};
    if (train && drop)
        for (int i = 0; i < 3; ++i) dmask[i] = drop[i];
    float* part = at<float>(ws, p.stat_part);

    auto finalize = [&](int l, int nblk) {
        const Layer& L = p.L[l];
        BnFwdArgs f{};
        f.C = L.cout;
        f.nblk = nblk;
        f.part0 = part;
        f.part1 = part + (size_t)L.cout * nblk;
        f.partn = part + (size_t)2 * L.cout * nblk;
        f.gamma = P[p_bn_g(l)];
        f.beta = P[p_bn_b(l)];
        f.bias = P[p_conv_b(l)];
        f.rmean = bnstat[2 * (l - 1)];
        f.rvar = bnstat[2 * (l - 1) + 1];
        f.nbt = nbt ? nbt[l - 1] : nullptr;
        f.momentum = mom;
        f.eps = eps;
        f.train = train;
        f.cf = at<float4>(ws, L.cf);
        Scope sc(&p.prof, s, "bn_fwd_finalize");
        return launch_bn_fwd_finalize(f, s);
    };

    // layer 1: Cin = 1 direct conv
    {
        const Layer& L = p.L[1];
        Conv1Args c{};
        c.B = B; c.H = L.H; c.W = L.W; c.cout = L.cout;
        c.x = x;
        c.w = P[p_conv_w(1)];
        c.out = at<float>(ws, L.y);
        c.part0 = part;
        c.part1 = part + (size_t)L.cout * L.nblk;
        c.partn = part + (size_t)2 * L.cout * L.nblk;
        c.nblk = L.nblk;
        c.rows_per_blk = p.conv1_rows;
        { Scope sc(&p.prof, s, "conv1_fwd", 1); RC(launch_conv1_fwd(c, s)); }
        RC(finalize(1, L.nblk));
    }
    {  // the Winograd layers' transformed weights, all in one launch
        WinoPackJobs j{};
        for (int l = 2; l <= 6; ++l)
            if (p.L[l].wino) j.add(P[p_conv_w(l)], at<float>(ws, p.L[l].wu), p.L[l].cout, p.L[l].cin, 0);
        RC(launch_wino_pack_multi(j, s));
    }
    for (int l = 2; l <= 6; ++l) {
        const Layer& L = p.L[l];
        const Layer& Lp = p.L[l - 1];
        if (!L.wino) RC(launch_pack_fwd(P[p_conv_w(l)], at<float>(ws, L.wu), L.cout, L.cin, s));
        ConvArgs c{};
        c.B = B; c.H = L.H; c.W = L.W; c.cin = L.cin; c.cout = L.cout;
        c.src = at<float>(ws, Lp.y);
        c.cf_in = at<float4>(ws, Lp.cf);
        c.drop_in = L.pooled_in ? dmask[L.drop_idx] : nullptr;
        c.srcH = L.srcH; c.srcW = L.srcW;
        c.wpack = at<float>(ws, L.wu);
        c.out = at<float>(ws, L.y);
        c.part0 = part;
        c.part1 = part + (size_t)L.cout * L.nblk;
        c.partn = part + (size_t)2 * L.cout * L.nblk;
        c.nblk = L.wino ? L.nblk : (int)conv3x3_nblk(B, L.H, L.W, L.cout);
        c.src_guard = 1;  // workspace tensors (and the input never reaches a 3x3 conv)
        c.queue = p.wq ? at<int>(ws, p.wq) : nullptr;
        if (l < 6 && p.L[l + 1].psel) {  // this conv's epilogue also makes the next block tail's pool selection
            c.pool_gamma = P[p_bn_g(l)];
            c.pool_ysel = at<float>(ws, p.L[l + 1].ysel);
            c.pool_arg = at<uint8_t>(ws, p.L[l + 1].parg);
        }
        int pro = PRO_BNRELU;
        if (L.pooled_in && L.psel) {  // block tail from the producer's selection: one light pass over ysel
            Scope sc(&p.prof, s, "pool_act", l);
            RC(launch_pool_act(at<float>(ws, L.ysel), c.cf_in, c.drop_in, at<float>(ws, L.xp), B, L.cin, L.H * L.W, s));
            c.src = at<float>(ws, L.xp);
            c.srcH = L.H; c.srcW = L.W;
            pro = PRO_RAW;
        } else if (L.pooled_in) {  // block tail materialised once; the conv and its wgrad read it raw
            Scope sc(&p.prof, s, "bn_relu_pool", l);
            RC(launch_bn_relu_pool(c.src, c.cf_in, c.drop_in, at<float>(ws, L.xp), B, L.cin, L.srcH,
                                   L.srcW, s, L.ysel ? at<float>(ws, L.ysel) : nullptr,
                                   L.parg ? at<uint8_t>(ws, L.parg) : nullptr));
            c.src = at<float>(ws, L.xp);
            c.srcH = L.H; c.srcW = L.W;
            pro = PRO_RAW;
        }
        {
            Scope sc(&p.prof, s, "conv_fwd", l);
            RC(L.wino ? launch_conv3x3_wino(pro, EPI_FWD, c, s) : launch_conv3x3_dma(pro, EPI_FWD, c, s));
        }
        RC(finalize(l, c.nblk));
    }
    // head: attention + mean pool on x6 = Dropout2d(ReLU(BN6(y6)))
    const int ia = 24, ip = p.cfg.use_attention ? 26 : 24;
    {
        HeadPoolArgs h{};
        h.B = B; h.C = p.C6; h.P = p.P6;
        h.y = at<float>(ws, p.L[6].y);
        h.cf = at<float4>(ws, p.L[6].cf);
        h.drop = dmask[2];
        h.wa = p.cfg.use_attention ? P[ia] : nullptr;
        h.ba = p.cfg.use_attention ? P[ia + 1] : nullptr;
        h.pooled = at<float>(ws, p.pooled);
        h.att = at<float>(ws, p.att);
        { Scope sc(&p.prof, s, "head_pool_fwd"); RC(launch_head_pool_fwd(h, s)); }
    }
    {
        RC(launch_transpose(P[ip], at<float>(ws, p.wt), p.D, p.C6, s));
        ProjArgs j{};
        j.B = B; j.K = p.C6; j.D = p.D;
        j.pooled = at<float>(ws, p.pooled);
        j.w = P[ip];
        j.wt = at<float>(ws, p.wt);
        j.bias = P[ip + 1];
        j.gamma = P[ip + 2];
        j.beta = P[ip + 3];
        j.rmean = bnstat[12];
        j.rvar = bnstat[13];
        j.nbt = nbt ? nbt[6] : nullptr;
        j.momentum = mom;
        j.eps = eps;
        j.train = train;
        j.h = at<float>(ws, p.h);
        j.cf = at<float4>(ws, p.cfp);
        j.emb = emb;
        j.norm = at<float>(ws, p.norm);
        { Scope sc(&p.prof, s, "proj_fwd"); RC(launch_proj_fwd(j, s)); }
    }
    return PCX_OK;
}

int small_backward(const Plan& p, const float* const* P, const float* x, const float* const* drop,
                   const float* emb, const float* demb, float* const* G, void* ws, hipStream_t s) {
    const int B = p.B;
    if (p.wq) RC(hip_status_ok(hipMemsetAsync(at<int>(ws, p.wq), 0, WINO_QUEUE_INTS * 4, s), "memset queue"));
    const float* dmask[3] = {nullptr, nullptr, nullptr};
    if (drop)
        for (int i = 0; i < 3; ++i) dmask[i] = drop[i];
    float* part = at<float>(ws, p.stat_part);
    float* wgp = at<float>(ws, p.wg_part);
    const int ia = 24, ip = p.cfg.use_attention ? 26 : 24;
    p.buckets.begin();

    // projection / BN1d / normalize backward
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
        { Scope sc(&p.prof, s, "proj_bwd"); RC(launch_proj_bwd(j, s)); }
    }
    p.buckets.mark(ip, s);
    // attention + pool + Dropout2d + ReLU backward -> dz6 and BN6 partials
    {
        HeadPoolArgs h{};
        h.B = B; h.C = p.C6; h.P = p.P6;
        h.y = at<float>(ws, p.L[6].y);
        h.cf = at<float4>(ws, p.L[6].cf);
        h.drop = dmask[2];
        h.wa = p.cfg.use_attention ? P[ia] : nullptr;
        h.ba = p.cfg.use_attention ? P[ia + 1] : nullptr;
        h.att = at<float>(ws, p.att);
        h.dpooled = at<float>(ws, p.dpooled);
        h.dz = at<float>(ws, p.L[6].dz);
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
    auto bwd_finalize = [&](int l, int nblk, double count) {
        const Layer& L = p.L[l];
        BnBwdArgs f{};
        f.C = L.cout;
        f.nblk = nblk;
        f.count = count;
        f.part0 = part;
        f.part1 = part + (size_t)L.cout * nblk;
        f.gamma = P[p_bn_g(l)];
        f.cf_fwd = at<float4>(ws, L.cf);
        f.dgamma = G[p_bn_g(l)];
        f.dbeta = G[p_bn_b(l)];
        f.cf = at<float4>(ws, L.cfb);
        // conv l's bias feeds this train-mode BN: its exact gradient is zero (sum over b, h, w of the BN
        // backward), written here before layer l's weight gradient marks its bucket (no memset launch)
        f.zero = G[p_conv_b(l)];
        Scope sc(&p.prof, s, "bn_bwd_finalize");
        return launch_bn_bwd_finalize(f, s);
    };
    RC(bwd_finalize(6, B, (double)B * p.P6));
    {  // the flipped Winograd weights of every Winograd data gradient (fused or not), in one launch
        WinoPackJobs j{};
        for (int l = 6; l >= 2; --l)
            if (p.L[l].wgbd || p.L[l].wino) j.add(P[p_conv_w(l)], at<float>(ws, p.L[l].wud), p.L[l].cin, p.L[l].cout, 1);
        RC(launch_wino_pack_multi(j, s));
    }

    for (int l = 6; l >= 2; --l) {
        const Layer& L = p.L[l];
        const Layer& Lp = p.L[l - 1];
        if (L.wgbd) {  // ---- weight and data gradient in one pass (dy never materialised)
            WinoBwdArgs w = L.wb;
            w.B = B; w.H = L.H; w.W = L.W;
            w.dz = at<float>(ws, L.dz);
            if (L.pd) {  // layer 3's data gradient left dz2 pooled (EPI_BWD_POOLSELP): rebuilt while staging
                w.dz = nullptr;
                w.dzpool = at<float>(ws, L.dz);
                w.parg = at<uint8_t>(ws, p.L[3].parg);
            }
            w.y = at<float>(ws, L.y);
            w.cf_dy = at<float4>(ws, L.cfb);
            w.yp = at<float>(ws, Lp.y);
            w.cf_x = at<float4>(ws, Lp.cf);
            w.up = at<float>(ws, L.wud);
            w.part = wgp;
            w.dzp = at<float>(ws, Lp.dz);
            w.bn0 = part;
            w.bn1 = part + (size_t)Lp.cout * w.nslice;
            {
                Scope sc(&p.prof, s, "wgbd", l);
                RC(launch_wgbd_wino(w, s));
            }
            {
                Scope sc(&p.prof, s, "wgrad_reduce", l);
                RC(launch_wgrad_wino_reduce(wgp, w.nslice, L.cout, L.cin, G[p_conv_w(l)], s));
            }
            p.buckets.mark(p_conv_w(l), s);
            RC(bwd_finalize(l - 1, w.nslice, (double)B * Lp.H * Lp.W));
            continue;
        }
        // ---- weight gradient
        if (L.wgw) {
            WinoWgradArgs w = L.ww;
            w.B = B; w.H = L.H; w.W = L.W; w.cin = L.cin; w.cout = L.cout;
            w.dz = at<float>(ws, L.dz);
            if (L.pd) {  // the next layer's data gradient left dz pooled (EPI_BWD_POOLSELP): rebuilt while staging
                w.dz = nullptr;
                w.dzpool = at<float>(ws, L.dz);
                w.parg = at<uint8_t>(ws, p.L[l + 1].parg);
            }
            w.y = at<float>(ws, L.y);
            w.cf_dy = at<float4>(ws, L.cfb);
            w.src = L.pooled_in ? at<float>(ws, L.xp) : at<float>(ws, Lp.y);
            w.cf_x = at<float4>(ws, Lp.cf);
            w.part = wgp;
            w.dy_out = at<float>(ws, p.dyb);
            {
                Scope sc(&p.prof, s, "wgrad", l);
                RC(launch_wgrad_wino(L.pooled_in ? PRO_RAW : PRO_BNRELU, w, s));
            }
            {
                Scope sc(&p.prof, s, "wgrad_reduce", l);
                RC(launch_wgrad_wino_reduce(wgp, w.nslice, L.cout, L.cin, G[p_conv_w(l)], s));
            }
            p.buckets.mark(p_conv_w(l), s);
        } else {
            WgradArgs w = L.wg;
            w.B = B; w.H = L.H; w.W = L.W; w.cin = L.cin; w.cout = L.cout;
            w.dz = at<float>(ws, L.dz);
            w.y = at<float>(ws, L.y);
            w.cf_dy = at<float4>(ws, L.cfb);
            w.src = at<float>(ws, Lp.y);
            w.cf_x = at<float4>(ws, Lp.cf);
            w.drop = L.pooled_in ? dmask[L.drop_idx] : nullptr;
            w.srcH = L.srcH; w.srcW = L.srcW;
            w.part = wgp;
            int pro = PRO_BNRELU;
            if (L.pooled_in) {  // pooled input materialised by the forward
                w.src = at<float>(ws, L.xp);
                w.srcH = L.H; w.srcW = L.W;
                pro = PRO_RAW;
            }
            w.dy_out = at<float>(ws, p.dyb);
            {
                Scope sc(&p.prof, s, "wgrad", l);
                RC(launch_wgrad_s(pro, w, s));
            }
            { Scope sc(&p.prof, s, "wgrad_reduce", l); RC(launch_sum_slices(wgp, w.nslice, (int64_t)L.cout * L.cin * 9, G[p_conv_w(l)], s)); }
            p.buckets.mark(p_conv_w(l), s);  // BN l's dgamma / dbeta came with layer l+1's data gradient
        }
        // ---- data gradient -> dz of the previous BN (through ReLU / MaxPool / Dropout2d)
        {
            if (!L.wino) RC(launch_pack_dgrad(P[p_conv_w(l)], at<float>(ws, L.wud), L.cout, L.cin, s));
            float* dzp = at<float>(ws, Lp.dz);
            if (L.pooled_in && ((L.srcH & 1) || (L.srcW & 1)))
                RC(hip_status_ok(hipMemsetAsync(dzp, 0, (size_t)B * Lp.cout * L.srcH * L.srcW * 4, s),
                                 "memset dz"));
            ConvArgs c{};
            c.B = B; c.H = L.H; c.W = L.W; c.cin = L.cout; c.cout = L.cin;
            c.src = at<float>(ws, L.dz);
            c.src2 = at<float>(ws, L.y);
            c.cf_in = at<float4>(ws, L.cfb);
            c.src = at<float>(ws, p.dyb);  // dy = BN backward of (dz, y), materialised by the weight gradient
            c.src_guard = 1;
            c.queue = p.wq ? at<int>(ws, p.wq) : nullptr;
            c.srcH = L.H; c.srcW = L.W;
            c.wpack = at<float>(ws, L.wud);
            c.out = dzp;
            c.yprev = at<float>(ws, Lp.y);
            c.cf_out = at<float4>(ws, Lp.cf);
            c.drop_out = L.pooled_in ? dmask[L.drop_idx] : nullptr;
            c.Hs = L.srcH; c.Ws = L.srcW;
            const int nblk = L.wino ? L.nblk : (int)conv3x3_nblk(B, L.H, L.W, L.cin);
            c.part0 = part;
            c.part1 = part + (size_t)L.cin * nblk;
            c.nblk = nblk;
            {
                Scope sc(&p.prof, s, "conv_dgrad", l);
                // pooled input with a recorded selection: the epilogue reads it at the pooled resolution
                int epi = !L.pooled_in ? EPI_BWD_RELU : L.ysel ? EPI_BWD_POOLSEL : EPI_BWD_POOL;
                if (epi == EPI_BWD_POOLSEL) {
                    c.ysel = at<float>(ws, L.ysel);
                    c.parg = at<uint8_t>(ws, L.parg);
                    if (Lp.pd) {  // the previous layer's weight gradient rebuilds dz's windows itself
                        epi = EPI_BWD_POOLSELP;
                        c.dpool = dzp;
                    }
                }
                RC(L.wino ? launch_conv3x3_wino(PRO_RAW, epi, c, s) : launch_conv3x3_dma(PRO_RAW, epi, c, s));
            }
            RC(bwd_finalize(l - 1, nblk, (double)B * Lp.H * Lp.W));
        }
    }
    // layer 1 weight gradient (input has one channel)
    {
        const Layer& L = p.L[1];
        Wgrad1Args w{};
        w.B = B; w.H = L.H; w.W = L.W; w.cout = L.cout;
        w.dz = at<float>(ws, L.dz);
        w.y = nullptr;  // y1 recomputed from the input window (bit-identical to conv1_fwd's): dz1 alone streamed
        w.w = P[p_conv_w(1)];
        w.cf_dy = at<float4>(ws, L.cfb);
        w.x = x;
        w.part = wgp;
        w.nslice = p.wg1_nslice;
        w.rows_per_slice = p.wg1_rows;
        { Scope sc(&p.prof, s, "wgrad", 1); RC(launch_wgrad1(w, s)); }
        RC(launch_sum_slices(wgp, w.nslice, (int64_t)L.cout * 9, G[p_conv_w(1)], s));
    }
    p.buckets.mark(0, s);
    return PCX_OK;
}

}  // namespace pcx

// ====================================================================== C ABI
using pcx::Plan;

extern "C" void* pcx_net_create(const pcx_net_config* cfg, int64_t B, int64_t F, int64_t T) {
    using namespace pcx;
    if (!cfg) { set_error("pcx_net_create: NULL config"); return nullptr; }
    if (cfg->in_channels != 1) { set_error("pcx_net_create: in_channels must be 1 (MFCC input)"); return nullptr; }
    if (B < 1 || F < 1 || T < 1 || B * F * T > ((int64_t)1 << 40)) {
        set_error("pcx_net_create: bad input shape [%lld,1,%lld,%lld]", (long long)B, (long long)F, (long long)T);
        return nullptr;
    }
    if (cfg->embedding_dim < 1 || cfg->embedding_dim > 256) {
        set_error("pcx_net_create: embedding_dim %d unsupported (1..256)", cfg->embedding_dim);
        return nullptr;
    }
    Plan* p = new Plan();
    p->cfg = *cfg;
    p->B = (int)B; p->F = (int)F; p->T = (int)T; p->D = cfg->embedding_dim;
    p->total = 256;  // guard: every region has >= 256 readable workspace bytes in front of it (conv_wino X4)
    int rc = PCX_EINVAL;
    if (cfg->kind == PCX_NET_CNN_SMALL && cfg->conv_bf16)
        set_error("pcx_net_create: conv_bf16 is a PhonemeNetDeep option (cnn_small is float32)");
    else if (cfg->kind == PCX_NET_CNN_SMALL) rc = build_small(*p);
    else if (cfg->kind == PCX_NET_CNN_DEEP) rc = build_deep(*p);
    else set_error("pcx_net_create: network kind %d not supported", cfg->kind);
    if (rc) { delete p; return nullptr; }
    return p;
}

extern "C" void pcx_net_destroy(void* plan) { delete static_cast<Plan*>(plan); }

extern "C" size_t pcx_net_workspace_bytes(const void* plan) {
    return plan ? static_cast<const Plan*>(plan)->total : 0;
}

extern "C" int pcx_net_info(const void* plan, int* nparams, int* nbn, int* ndrop, int* drop_channels) {
    using namespace pcx;
    PCX_CHECK_ARG(plan, "pcx_net_info: NULL plan");
    const Plan* p = static_cast<const Plan*>(plan);
    if (nparams) *nparams = p->nparams;
    if (nbn) *nbn = p->nbn;
    if (ndrop) *ndrop = p->ndrop;
    if (drop_channels)
        for (int i = 0; i < p->ndrop; ++i) drop_channels[i] = p->drop_ch[i];
    return PCX_OK;
}

extern "C" int pcx_net_region(const void* plan, const char* name, size_t* offset, size_t* bytes) {
    using namespace pcx;
    PCX_CHECK_ARG(plan && name, "pcx_net_region: NULL argument");
    const Plan* p = static_cast<const Plan*>(plan);
    for (const auto& r : p->regions)
        if (r.name == name) {
            if (offset) *offset = r.off;
            if (bytes) *bytes = r.bytes;
            return PCX_OK;
        }
    set_error("pcx_net_region: no region '%s'", name);
    return PCX_EINVAL;
}

extern "C" int pcx_net_forward(const void* plan, const float* const* params, float* const* bn_stats,
                               int64_t* const* bn_counts, const float* x, const float* const* dropout,
                               int train, float* emb, void* ws, size_t ws_bytes, hipStream_t stream) {
    using namespace pcx;
    PCX_CHECK_ARG(plan && params && bn_stats && x && emb && ws, "pcx_net_forward: NULL argument");
    const Plan* p = static_cast<const Plan*>(plan);
    if (ws_bytes < p->total) { set_error("pcx_net_forward: workspace too small"); return PCX_EWORKSPACE; }
    if (train && p->B < 2) {
        set_error("Expected more than 1 value per channel when training, got input size [1, %d]", p->D);
        return PCX_EINVAL;
    }
    if (p->deep) return deep_forward(*p, params, bn_stats, bn_counts, x, dropout, train, emb, ws, stream);
    return small_forward(*p, params, bn_stats, bn_counts, x, dropout, train, emb, ws, stream);
}

extern "C" int pcx_net_backward(const void* plan, const float* const* params, const float* x,
                                const float* const* dropout, const float* emb, const float* d_emb,
                                float* const* grads, void* ws, size_t ws_bytes, hipStream_t stream) {
    using namespace pcx;
    PCX_CHECK_ARG(plan && params && x && emb && d_emb && grads && ws, "pcx_net_backward: NULL argument");
    const Plan* p = static_cast<const Plan*>(plan);
    if (ws_bytes < p->total) { set_error("pcx_net_backward: workspace too small"); return PCX_EWORKSPACE; }
    if (p->deep) return deep_backward(*p, params, x, dropout, emb, d_emb, grads, ws, stream);
    return small_backward(*p, params, x, dropout, emb, d_emb, grads, ws, stream);
}

extern "C" int pcx_net_grad_buckets(void* plan, int n, const int* first_param) {
    using namespace pcx;
    PCX_CHECK_ARG(plan && n >= 0 && (n == 0 || first_param), "pcx_net_grad_buckets: bad argument");
    Plan* p = static_cast<Plan*>(plan);
    for (int k = 0; k < n; ++k) {
        const int hi = k ? first_param[k - 1] : p->nparams;
        PCX_CHECK_ARG(first_param[k] >= 0 && first_param[k] < hi, "pcx_net_grad_buckets: first_param[%d] = %d not in [0, %d)",
                      k, first_param[k], hi);
    }
    PCX_CHECK_ARG(n == 0 || first_param[n - 1] == 0, "pcx_net_grad_buckets: the last bucket must start at parameter 0");
    p->buckets.clear();
    for (int k = 0; k < n; ++k) {
        hipEvent_t e;
        hipError_t err = hipEventCreateWithFlags(&e, hipEventDisableTiming);
        if (err != hipSuccess) {
            p->buckets.clear();
            return hip_status(err, "pcx_net_grad_buckets");
        }
        p->buckets.ev.push_back(e);
        p->buckets.first.push_back(first_param[k]);
    }
    p->buckets.fired.assign(n, 0);
    return PCX_OK;
}

extern "C" int pcx_net_bucket_wait(void* plan, int k, hipStream_t stream) {
    using namespace pcx;
    PCX_CHECK_ARG(plan, "pcx_net_bucket_wait: NULL plan");
    Plan* p = static_cast<Plan*>(plan);
    PCX_CHECK_ARG(k >= 0 && k < (int)p->buckets.ev.size(), "pcx_net_bucket_wait: bucket %d of %d", k,
                  (int)p->buckets.ev.size());
    PCX_CHECK_ARG(p->buckets.fired[k], "pcx_net_bucket_wait: bucket %d was not recorded by a backward", k);
    return hip_status_ok(hipStreamWaitEvent(stream, p->buckets.ev[k], 0), "pcx_net_bucket_wait");
}

extern "C" int pcx_net_grad_stages(const void* plan, int* first_param, int max_entries) {
    using namespace pcx;
    PCX_CHECK_ARG(plan, "pcx_net_grad_stages: NULL plan");
    const Plan* p = static_cast<const Plan*>(plan);
    const int n = (int)p->stages.size();
    for (int i = 0; i < n && i < max_entries; ++i)
        if (first_param) first_param[i] = p->stages[i];
    return n;
}

extern "C" int pcx_net_profile(void* plan, int enable) {
    using namespace pcx;
    PCX_CHECK_ARG(plan, "pcx_net_profile: NULL plan");
    Plan* p = static_cast<Plan*>(plan);
    p->prof.clear();
    p->prof.on = enable != 0;
    return PCX_OK;
}

extern "C" int pcx_net_profile_only(void* plan, const char* label) {
    using namespace pcx;
    PCX_CHECK_ARG(plan, "pcx_net_profile_only: NULL plan");
    static_cast<Plan*>(plan)->prof.only = label ? label : "";
    return PCX_OK;
}

extern "C" int pcx_net_profile_read(void* plan, char* labels, size_t labels_len, float* total_ms,
                                    int* counts, int max_entries) {
    using namespace pcx;
    PCX_CHECK_ARG(plan, "pcx_net_profile_read: NULL plan");
    Plan* p = static_cast<Plan*>(plan);
    std::vector<std::string> names;
    std::vector<double> tot;
    std::vector<int> cnt;
    for (size_t i = 0; i < p->prof.spans.size(); ++i) {
        float ms = 0.f;
        hipError_t e = hipEventSynchronize(p->prof.spans[i].second);
        if (e != hipSuccess) return hip_status(e, "pcx_net_profile_read");
        (void)hipEventElapsedTime(&ms, p->prof.spans[i].first, p->prof.spans[i].second);
        size_t k = 0;
        while (k < names.size() && names[k] != p->prof.labels[i]) ++k;
        if (k == names.size()) { names.push_back(p->prof.labels[i]); tot.push_back(0.0); cnt.push_back(0); }
        tot[k] += ms;
        cnt[k] += 1;
    }
    std::string joined;
    int n = 0;
    for (size_t k = 0; k < names.size() && (int)k < max_entries; ++k, ++n) {
        if (total_ms) total_ms[k] = (float)tot[k];
        if (counts) counts[k] = cnt[k];
        joined += names[k];
        joined += '\n';
    }
    if (labels && labels_len) {
        size_t c = std::min(joined.size(), labels_len - 1);
        memcpy(labels, joined.data(), c);
        labels[c] = 0;
    }
    p->prof.clear();
    return n;
}
