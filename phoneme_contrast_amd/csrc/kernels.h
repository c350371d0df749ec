// Internal (C++) launch interface shared by the kernel files and the network orchestrator.
// Not part of the C ABI.  All tensors are fp32, planar NCHW (the reference's own layout).
#pragma once
#include "pcx_common.h"

namespace pcx {

// ------------------------------------------------------------------ prologue / epilogue kinds
// What a conv kernel applies to its input while staging it into LDS:
enum Prologue {
    PRO_RAW = 0,        // x = src
    PRO_BNRELU = 1,     // x = max(0, src*s[c] + t[c])                        (cf = {s,t,.,.})
};
// What a conv kernel does with its accumulator tile:
enum Epilogue {
    EPI_FWD = 0,        // store y, per-block BN statistics (sum, M2, count)
    EPI_BWD_RELU = 1,   // dz = acc * [yprev*s+t > 0]; store dz; sums of dz and dz*xhat
    EPI_BWD_POOL = 2,   // route acc (pooled res) through dropout, 2x2 argmax, ReLU to 2x res
    EPI_BWD_STORE = 3,  // dx = acc (or dx += acc with ConvArgs::accumulate); no statistics
    EPI_BWD_POOLSEL = 4,  // EPI_BWD_POOL from the forward's recorded window selection (ysel / parg at the
                          // pooled resolution: no full-resolution window reads; conv_wino only)
    EPI_BWD_POOLSELP = 5, // EPI_BWD_POOLSEL writing the routed gradient at the pooled resolution (dpool):
                          // the consumer (wgbd_wino) rebuilds dz's 2x2 windows from parg
};

// 3x3 / stride 1 / pad 1 convolution as an implicit GEMM on v_mfma_f32_32x32x2_f32.
// Used for the forward pass (weights packed [9][cin][cout]) and for the data gradient
// (dy in, dx out, weights packed flipped [9][cout_fwd][cin_fwd]).
struct ConvArgs {
    int B, H, W;          // conv resolution (input == output for stride 1, pad 1)
    int cin, cout;        // GEMM channels (dgrad: cin = dy channels, cout = dx channels)
    // prologue source
    const float* src;
    const float* src2;
    const float4* cf_in;
    const float* drop_in;
    int srcH, srcW;
    const float* wpack;   // [9][cin][cout]
    // epilogue
    float* out;
    const float* yprev;
    const float4* cf_out; // EPI_BWD_*: {s, t, mean, invstd} of the BN feeding the prologue
    const float* drop_out;
    int Hs, Ws;           // EPI_BWD_POOL: resolution of dz (2H or 2H+1, ...)
    float* part0;         // [cout][nblk] statistics partials
    float* part1;
    float* partn;         // [nblk] element counts (EPI_FWD)
    int nblk;
    int NR, RS;           // staged rows / LDS row stride (host-computed)
    int accumulate;       // EPI_BWD_STORE: add into out instead of overwriting
    int src_guard;        // 1: at least 4 readable bytes precede src (conv_wino's 16-byte staging copies)
    const float* ysel;    // EPI_BWD_POOLSEL: y at each 2x2 window's selected element [B][cout][H][W] (pooled res)
    const uint8_t* parg;  // EPI_BWD_POOLSEL: the selected element (0..3, row-major) of each window
    float* dpool;         // EPI_BWD_POOLSELP: the routed gradient at the pooled resolution [B][cout][H][W]
    int* queue;           // conv_wino: unit queue (WINO_QUEUE_INTS, zero before the first launch; each launch
                          // leaves it zero), nullptr = static unit order
    // conv_wino EPI_FWD (optional, round 6): also the next block's 2x2 max-pool selection of relu(BN(y)) -- y at
    // each window's selected element and its index at the pooled resolution [B][cout][H / 2][W / 2] -- from
    // the sign of that BN's gamma (the selection bn_relu_pool_kernel records)
    const float* pool_gamma;
    float* pool_ysel;
    uint8_t* pool_arg;
};
constexpr int WINO_QUEUE_INTS = 9 * 32;  // 8 per-XCD unit counters + a completion counter, 128 B apart

size_t conv3x3_nblk(int B, int H, int W, int cout);
// Raw rows DMA'd into LDS (global_load_lds, double-buffered), the prologue applied at operand-read
// time (conv_dma.hip).  Prologues PRO_RAW, PRO_BNRELU.
int launch_conv3x3_dma(int pro, int epi, ConvArgs a, hipStream_t s);
// Winograd F(2x2, 3x3) form of the same conv (conv_wino.hip): same ConvArgs / prologues /
// epilogues, weights transformed by launch_wino_pack into U = G g G^T, packed
// [cout / 32][cin][4][32][4].  Partials are per 64-tile block: nblk = wino_nblk().
struct WinoGeo {
    int TR, TC, NTS, BPS;  // tile rows / columns per sample, tiles per sample, 64-tile blocks per sample
    int ncg;               // output-channel groups of 32
    float inv_ncg, inv_BPS, inv_TC;  // reciprocals for the kernel's unit decode
    int naive_slots;                 // analysis: blockIdx order instead of the XCD-contiguous one (PCX_WINO_SLOT=1)
    int span;                        // units of 64 consecutive tiles of the whole batch (narrow images)
    int NTOT, nblk;                  // B * NTS; 64-tile blocks (BN partials) of the launch
    float inv_NTS, inv_TR;
};
bool wino_geometry(int B, int H, int W, int cin, int cout, WinoGeo* g);
// Narrow images (W < 31, the 5 x 25 / 3 x 13 blocks of cnn_deep): units span rows and samples (a wave's 16
// tiles in up to 4 row segments side by side in its slot).  PRO_RAW with EPI_FWD / EPI_BWD_STORE, 16-byte
// staging only (ConvArgs::src_guard), cin % 8 == 0.
bool wino_span_geometry(int B, int H, int W, int cin, int cout, WinoGeo* g);
size_t wino_nblk(int B, int H, int W, int cin, int cout);
// flip = 0: forward weights w[M][K][3][3]; flip = 1: data gradient of forward weights w[K][M][3][3]
int launch_wino_pack(const float* w, float* u, int M, int K, int flip, hipStream_t s);
struct WinoPackJobs {  // up to MAXJ launch_wino_pack calls in one launch
    static constexpr int MAXJ = 8;
    int n;
    const float* w[MAXJ];
    float* u[MAXJ];
    int M[MAXJ], K[MAXJ], flip[MAXJ];
    void add(const float* w_, float* u_, int M_, int K_, int flip_) {
        w[n] = w_; u[n] = u_; M[n] = M_; K[n] = K_; flip[n] = flip_; ++n;
    }
};
int launch_wino_pack_multi(const WinoPackJobs& j, hipStream_t s);
int launch_conv3x3_wino(int pro, int epi, ConvArgs a, hipStream_t s);
// materialised block tail x = drop * maxpool2(relu(y*s + t)) (feeds PRO_RAW convs)
// ysel / parg (optional, both or neither): y at each window's first maximum of relu(y s + t) (torch's
// max_pool2d rule) and its index, for the EPI_BWD_POOLSEL data gradient
int launch_bn_relu_pool(const float* y, const float4* cf, const float* drop, float* x, int B, int C,
                        int Hs, int Ws, hipStream_t s, float* ysel = nullptr, uint8_t* parg = nullptr);
// the same block tail from a selection made by the producer conv (ConvArgs::pool_ysel): x = drop * relu(ysel s + t)
// over [B][C][HWp] (HWp % 4 == 0)
int launch_pool_act(const float* ysel, const float4* cf, const float* drop, float* x, int B, int C, int HWp,
                    hipStream_t s);

// Cin = 1 convolution (first layer), 3x3 pad 1, with BN statistics.
struct Conv1Args {
    int B, H, W, cout;
    const float* x;       // [B][1][H][W]
    const float* w;       // [cout][1][3][3] (reference layout)
    float* out;           // [B][cout][H][W]
    float* part0;
    float* part1;
    float* partn;
    int nblk, rows_per_blk;
};
int launch_conv1_fwd(Conv1Args a, hipStream_t s);
int conv1_nblk(int B, int H, int* rows_per_blk);

// Weight gradient of a 3x3 conv: dW[n][c][tap] = sum dy[n] * x[c](shifted), dy = BNBWD(dz, y),
// x = prologue(src) exactly as in the forward conv.  Partials per slice, then summed.
struct WgradArgs {
    int B, H, W, cin, cout;
    const float* dz;
    const float* y;
    const float4* cf_dy;  // {a, mb, mgi, mean}
    const float* src;
    const float4* cf_x;
    const float* drop;
    int srcH, srcW;
    float* part;          // [nslice][cout][cin][9]
    float* dy_out;        // optional: dy = BNBWD(dz, y) written here (consumed by the data grad)
    int R, CW, nseg, nrb, nchunks, per_slice, nslice;
    int MT, NPM, NPC;     // MFMA tile (16 or 32), tiles per block along cout / cin
    int VX;               // vector width of the staged loads
    int KW, ntslice;      // wgrad_w32: waves splitting K on one tile, task slices (nslice = ntslice * KW)
    int R0, DCS, XCS;     // wgrad_s: stream length, LDS channel strides of dy / x
    int nvd, nvx;         // wgrad_s: staged vectors per dy / x channel row
};
// sliding row window on 32 x 32 tiles (wgrad_w32.hip; channels multiples of 32; the narrow-row residual
// convs): false if it does not apply
bool wgrad_w32_geometry(int B, int H, int W, int cin, int cout, WgradArgs* a);
int launch_wgrad_w32(int pro, WgradArgs a, hipStream_t s);
// pixel-stream kernel (wgrad_s.hip, 16x16x4 tiles): channels multiples of 32, any W; force_cw > 0 pins the
// strip width (timing tools)
bool wgrad_s_geometry(int B, int H, int W, int cin, int cout, WgradArgs* a, int force_cw = 0);
int launch_wgrad_s(int pro, WgradArgs a, hipStream_t s);

// Winograd F(2x2,3x3) weight gradient of the stride-1 3x3 convs (wgrad_wino.hip): 32 x 32 channel
// blocks, column strips of <= 50 tiles, W a multiple of 2; false if it does not apply
struct WinoWgradArgs {
    int B, H, W, cin, cout;
    const float* dz;
    const float* dzpool;  // (instead of dz, optional) behind a 2x2 MaxPool: the routed gradient at the pooled
    const uint8_t* parg;  //   resolution + the window selection (conv_wino EPI_BWD_POOLSELP); dz rebuilt
    const float* y;
    const float4* cf_dy;  // {a, mb, mgi, mean}: dy = BN backward of (dz, y)
    const float* src;     // x (raw, or the producer's y under PRO_BNRELU)
    const float4* cf_x;
    float* part;          // [nslice][cout][cin][16] Winograd-domain partials
    float* dy_out;        // optional: dy written here by the cin-group-0 blocks
    int S, nseg, V, XCS, DCS, nd, nx, Ksteps;  // strip tiles, strips per row, vector width, LDS strides, items
    int NH;               // input-channel halves per block (2: 64 input channels, 8 waves)
    size_t lds;
    int ntask, per_slice, nslice;
};
bool wgrad_wino_geometry(int B, int H, int W, int cin, int cout, WinoWgradArgs* a);
int launch_wgrad_wino(int pro, WinoWgradArgs a, hipStream_t s);
// dW [cout][cin][3][3] = G^T (sum of the slices) G, float64, fixed order
int launch_wgrad_wino_reduce(const float* part, int nslice, int cout, int cin, float* dw, hipStream_t s);

// cnn_small layer-2 backward in one kernel (wgbd_wino.hip): Winograd weight gradient AND data gradient of
// a 32 -> 32 stride-1 3x3 conv from one staging of dz, y (dy = BN backward) and y_prev (x = relu(BN_prev)),
// with the producer's ReLU mask and BN backward sums in the data gradient's epilogue (EPI_BWD_RELU)
struct WinoBwdArgs {
    int B, H, W;           // 32 channels in and out; W % 4 == 0, W / 2 even
    const float* dz;       // [B][32][H][W] gradient of this conv's BN output
    const float* dzpool;   // (instead of dz, optional) behind a 2x2 MaxPool: the routed gradient at the
    const uint8_t* parg;   //   pooled resolution [B][32][H/2][W/2] and the window selection (conv_wino's
                           //   EPI_BWD_POOLSELP / bn_relu_pool); dz is rebuilt while staging
    const float* y;        // [B][32][H][W] raw conv output
    const float4* cf_dy;   // {a, mb, mgi, mean}: dy = a (dz - mb - (y - mean) mgi)
    const float* yp;       // [B][32][H][W] producer's raw output: x = relu(s yp + t)
    const float4* cf_x;    // producer BN forward coefficients {s, t, mean, invstd}
    const float* up;       // U' of the flipped weights: launch_wino_pack(w, up, 32, 32, 1)
    float* part;           // weight-gradient partials [nslice][32][32][16] (launch_wgrad_wino_reduce)
    float* dzp;            // out: [B][32][H][W] gradient of the producer BN's output
    float* bn0;            // out: [32][nslice] sum dzp
    float* bn1;            // out: [32][nslice] sum dzp * xhat_prev
    int nseg, seg_t0[4], seg_S[4];  // column strips (tiles) of a tile row
    int V, NIR, XCS;
    size_t lds;
    int ntask, per_slice, nslice;
    int paired;            // the two strips of a sample on two blocks of one XCD at the same time
};
bool wgbd_wino_geometry(int B, int H, int W, int C, WinoBwdArgs* a);
int launch_wgbd_wino(WinoBwdArgs a, hipStream_t s);

// PhonemeNetDeep 7x7 stem (Cin = 1, pad 3): direct forward + BN partials, weight gradient with the
// BN backward of (dz, y) in its loads (conv.hip)
struct StemArgs {
    int B, H, W, cout;
    const float* x;       // [B][1][H][W]
    const float* w;       // [cout][1][7][7]
    float* out;           // forward: y [B][cout][H][W]
    float* part0;         // forward: BN partials [cout][nblk] (sum, M2), counts [nblk]
    float* part1;
    float* partn;
    const float* dz;      // weight gradient: dz0, y0 and the BN-backward coefficients
    const float* y;
    const float4* cf_dy;
    float* part;          // weight gradient: [nblk slices][cout][49]
    int nblk, rows_per_blk;
    // fused bf16 stem (y0 recomputed instead of stored): MaxPool(3,2,1)(ReLU(BN0(y0))) outputs
    const float4* cf;     // BN0 forward coefficients {scale, shift, mean, istd}
    float* pool;          // (unused by the fused pool: a0 = relu(BN0(pool_ysel)) where needed)
    uint8_t* pool_arg;    // first-max tap per window (255: window max <= 0), pooled NHWC [B][OH][OW][cout]
    float* pool_ysel;     // y0 at the selected tap, pooled NHWC (BN0 backward xhat input; block 0 residual)
    void* pool_nhwc;      // optional: padded NHWC bf16 image of a0 [B][OH + 2][OW + 2][cout]
    int OH, OW;
    // fused backward: gradient of a0 in, dz0 (bf16, [B][cout][H][W]) out + BN0 backward sums, which the
    // recomputing weight gradient then reads (dz16)
    const float* dpool;
    const float* dpool2;  // optional second addend of the a0 gradient (block 0's identity shortcut)
    uint16_t* dz16;
    float* p_g;           // [cout][nslice] sums of dz0 and of dz0 * xhat
    float* p_x;
};
int stem_nblk(int B, int H, int* rows_per_blk);
int stem_wgrad_nslice(int B, int H, int* rows_per_slice, bool mfma = false);
bool stem_wgrad_mfma_ok(int cout, int H, int W);  // the MFMA weight-gradient forms (bf16 / fp32) apply
// fused bf16 stem: forward statistics only (a.out = nullptr), then the pooled outputs from a
// recomputed y0; weight gradient from dz0 and a recomputed y0 (no y0 plane anywhere)
bool stem_fused_ok(int cout, int H, int W);
int launch_stem_pool(StemArgs a, hipStream_t s);
int launch_stem_wgrad_rc(StemArgs a, hipStream_t s);
// MaxPool(3,2,1) + ReLU backward of the fused stem: dz0 (bf16) and the BN0 backward sums per (cout, slice)
int launch_stem_pool_bwd(StemArgs a, int* nslice, hipStream_t s);
int launch_stem_fwd(StemArgs a, int bf16, float* wround, hipStream_t s);  // wround: [cout][49] scratch (bf16)
int launch_stem_wgrad(StemArgs a, int bf16, hipStream_t s);

// first-layer (Cin = 1) weight gradient
struct Wgrad1Args {
    int B, H, W, cout;
    const float* dz;
    const float* y;       // the conv's output, or nullptr with w set: recomputed from x (bit-identical)
    const float* w;       // [cout][9] conv weights (y == nullptr)
    const float4* cf_dy;
    const float* x;
    float* part;          // [nslice][cout][9]
    int nslice, rows_per_slice;
};
int launch_wgrad1(Wgrad1Args a, hipStream_t s);
// slices of the layer-1 weight gradient for its kernel (rows_per_slice out; nslice returned)
int wgrad1_nslice(int B, int H, int W, int cout, int* rows_per_slice);

// sum `nslice` partial copies of an n-element array into out (deterministic order)
int launch_sum_slices(const float* part, int nslice, int64_t n, float* out, hipStream_t s);

// weight packing (reference layout [cout][cin][3][3])
int launch_pack_fwd(const float* w, float* wp, int cout, int cin, hipStream_t s);   // -> [9][cin][cout]
int launch_pack_dgrad(const float* w, float* wp, int cout, int cin, hipStream_t s); // -> [9][cout][cin] flipped

// ------------------------------------------------------------------ batch norm finalisers
struct BnFwdArgs {
    int C, nblk;
    const float* part0;   // sums   [C][nblk]
    const float* part1;   // M2     [C][nblk]
    const float* partn;   // counts [nblk]
    const float* gamma;
    const float* beta;
    const float* bias;    // conv bias (excluded from the stored raw output) or NULL
    float* rmean;
    float* rvar;
    int64_t* nbt;
    float momentum, eps;
    int train;
    float4* cf;           // out {s, t, mean, invstd}
};
int launch_bn_fwd_finalize(BnFwdArgs a, hipStream_t s);

struct BnBwdArgs {
    int C, nblk;
    double count;
    const float* part0;   // sum dz
    const float* part1;   // sum dz*xhat
    const float* gamma;
    const float4* cf_fwd; // {s, t, mean, invstd}
    float* dgamma;
    float* dbeta;
    float4* cf;           // out {a, mb, mgi, mean}
    float* zero;          // or NULL: C floats set to 0 (the producing conv's bias gradient: exactly 0 before a
                          // train-mode BN), instead of a memset launch
};
int launch_bn_bwd_finalize(BnBwdArgs a, hipStream_t s);

}  // namespace pcx

namespace pcx {

// ------------------------------------------------------------------ embedding head
// SpatialAttention + AdaptiveAvgPool2d(1) (reference phoneme_cnn.py:113-117,129-143) applied to
// x = drop * relu(y*s + t) (the last BN/ReLU/Dropout2d of the trunk, fused).
struct HeadPoolArgs {
    int B, C, P;
    const float* y;        // [B][C][P] raw conv output
    const float4* cf;      // {s, t, mean, invstd}
    const float* drop;     // [B][C] or NULL (NHWC_ACT: dropout of the result; NHWC_BNBWD: of the mask below)
    const float4* mcf;     // NHWC_BNBWD (optional): src is re-masked first, src drop [y mcf.x + mcf.y > 0]
                           // (the ReLU / Dropout2d backward bwd_prep_kernel applied without storing it)
    const float* wa;       // [C] attention 1x1 conv weight, NULL = no attention
    const float* ba;       // [1]
    float* pooled;         // [B][C]
    float* att;            // [B][P] sigmoid map (saved for backward)
    // backward
    const float* dpooled;  // [B][C]
    float* dz;             // [B][C][P]
    float* p_dz;           // [C][B]
    float* p_dzx;          // [C][B]
    float* p_dwa;          // [C][B]
    float* p_dba;          // [B]
};
int launch_head_pool_fwd(HeadPoolArgs a, hipStream_t s);
int launch_head_pool_bwd(HeadPoolArgs a, hipStream_t s);

// projection Linear(K -> D) + BatchNorm1d(D) + F.normalize (phoneme_cnn.py:75-77,119-124)
struct ProjArgs {
    int B, K, D;
    const float* pooled;   // [B][K]
    const float* w;        // [D][K] (reference layout)
    const float* wt;       // [K][D] packed transpose
    const float* bias;     // [D]
    const float* gamma;
    const float* beta;
    float* rmean;
    float* rvar;
    int64_t* nbt;
    float momentum, eps;
    int train;
    float* h;              // [B][D] linear output
    float4* cf;            // [D] {s, t, mean, invstd}
    float* emb;            // [B][D]
    float* norm;           // [B]
    // backward
    const float* demb;     // [B][D]
    float* dzp;            // [B][D]
    float4* cfb;           // [D] {a, mb, mgi, mean}
    float* dh;             // [B][D]
    float* dpooled;        // [B][K]
    float* dw;             // [D][K]
    float* db;             // [D]
    float* dgamma;
    float* dbeta;
    float* part;           // [proj_part_floats] weight / bias gradient partials
};
int proj_wg_nslice(int B);
size_t proj_part_floats(int B, int D, int K);
int launch_proj_fwd(ProjArgs a, hipStream_t s);
int launch_proj_bwd(ProjArgs a, hipStream_t s);
int launch_transpose(const float* in, float* out, int rows, int cols, hipStream_t s);

// out[r] = sum_c part[r][c] (float64, fixed order)
int launch_row_sum(const float* part, int rows, int64_t cols, float* out, hipStream_t s);

// ------------------------------------------------------------------ residual network (convg.hip)
// General KxK / stride 1|2 conv as an implicit GEMM: mode 0 forward, 1 data grad, 2 weight grad.
struct ConvGArgs {
    int mode;
    int B, cin, cout;
    int IH, IW, OH, OW;   // input / output resolution of the forward conv
    int KH, KW, stride, pad;
    const float* x;       // modes 0, 2: [B][cin][IH][IW]
    const float* w;       // modes 0, 1: [cout][cin][KH][KW] (reference layout)
    const float* dy;      // modes 1, 2: [B][cout][OH][OW]
    float* out;           // 0: y [B][cout][OH][OW]; 1: dx [B][cin][IH][IW]; 2: [nslice][cout][cin*KH*KW]
    int accumulate;       // modes 1, 3: dx += result
    int par;              // mode 3 (internal): parity class (ih % 2) * 2 + (iw % 2)
    int64_t kslice;       // mode 2: pixels per slice (multiple of 32)
    int nslice;
    int bf16;             // operands rounded to bf16, float32 accumulation (convg_bf16.hip)
    void* wpack;          // modes 0/1/3 (optional): scratch for the weights packed as GEMM rows
                          // (fp32 [M][K rounded to 16]; bf16 [M][K rounded to 32])
    // mode 2 only: dy computed while staging as BN backward of (bn_g, bn_y) with per-channel
    // {a, mb, mgi, mean} (dy = a (g - mb - (y - mean) mgi)); `dy` is then unused
    const float* bn_g;
    const float* bn_y;
    const float4* bn_cf;
    // mode 0 on the channel-last engine (optional): the BN forward partials of out in the epilogue --
    // per 128-pixel tile tn and channel c: st_part0[c][ntile] = sum, st_part1 = M2 about the tile mean,
    // st_partn[tn] = valid pixels; ntile = ceil(B OH OW / 128) (launch_bn_fwd_finalize's layout)
    float* st_part0;
    float* st_part1;
    float* st_partn;
    // mode 1 (stride 1) on the channel-last engine (optional): the backward partials of the BN + ReLU
    // (+ Dropout2d) feeding this conv's input, from out = dx in the epilogue (bwd_prep's MASK_BN sums):
    // g = dx ep_drop[b,c] [ep_y s + t > 0] (ep_cf = {s, t, mean, invstd}), per 128-pixel tile
    // ep_pg[c][ntile] = sum g, ep_px[c][ntile] = sum g (ep_y - mean) invstd; ntile = ceil(B IH IW / 128)
    const float* ep_y;
    const float4* ep_cf;
    const float* ep_drop;
    float* ep_pg;
    float* ep_px;
    // bf16 only: zero-padded channel-last bf16 images [B][H + 2][W + 2][C] of x (modes 0, 2) and dy
    // (modes 1, 2) written by launch_to_nhwc; when set, the channel-last engine (convn.hip) runs
    const void* xn;
    const void* dyn;
    // mode 1 stride 2, fp32 or the channel-last engine (optional): the four parity classes are written
    // dense, class-planar, into par_out (class q at par_off(q), [B][cin][IHc][IWc] each; together the
    // size of dx) instead of every other element of dx; launch_par_interleave then writes dx
    float* par_out;
};
// offset of parity class q's dense planes inside a class-planar buffer (see ConvGArgs::par_out)
int64_t par_off(int B, int C, int IH, int IW, int q);
// dx[b][c][ih][iw] (=|+=) class-planar src (classes of (ih % 2, iw % 2))
int launch_par_interleave(const float* src, float* dx, int B, int C, int IH, int IW, int accumulate, hipStream_t s);
// NCHW float32 -> zero-padded NHWC bf16 (convn.hip), optionally through the BN backward or the
// BN + residual + ReLU + dropout activation on the way
enum NhwcOp {
    NHWC_COPY = 0,   // src
    NHWC_BNBWD = 1,  // a (src - mb - (y - mean) mgi), cf = {a, mb, mgi, mean}
    NHWC_ACT = 2,    // drop[b,c] relu(src s + t + res'), res' = res rs + rt (rcf) | res | 0; cf = {s, t}
};
struct NhwcArgs {
    int op;
    int B, C, H, W;
    const float* src;
    const float* y;        // NHWC_BNBWD
    const float4* cf;
    const float* res;      // NHWC_ACT (optional)
    const float4* rcf;
    int res_pool;          // NHWC_ACT: res is the fused stem's y0 at the taps, pooled NHWC [B][H][W][C];
                           // residual term relu(res rs + rt) (= a0, rcf = the stem BN's coefficients)
    const float* drop;     // [B][C] or NULL (NHWC_ACT: dropout of the result; NHWC_BNBWD: of the mask below)
    const float4* mcf;     // NHWC_BNBWD (optional): src is re-masked first, src drop [y mcf.x + mcf.y > 0]
                           // (the ReLU / Dropout2d backward bwd_prep_kernel applied without storing it)
    float* out32;          // NHWC_ACT: optional float32 NCHW copy of the result
    uint8_t* mask8;        // NHWC_ACT: optional NCHW bytes [result > 0] (the backward's ReLU mask)
    void* dst;             // [B][H + 2][W + 2][C] bf16
    // NHWC_BNBWD (optional): a second image from the same src through a second BN backward (the
    // shortcut BN of a residual block shares the upstream gradient: read once, two images written)
    const float* y_b;
    const float4* cf_b;
    void* dst_b;
    int rows;              // (set by launch_to_nhwc) image rows per step
};
size_t nhwc_bytes(int B, int C, int H, int W);
int launch_to_nhwc(NhwcArgs a, hipStream_t s);
bool convn_fits(const ConvGArgs& a);
int64_t convn_stat_tiles(const ConvGArgs& a);  // mode 0: the st_part* tile count; mode 1: ep_p*
int64_t convn_tile_bound(int B, int H, int W);  // upper bound of convn_stat_tiles at an H x W resolution
int launch_convn(const ConvGArgs& a, hipStream_t s);
size_t convg_bf16_wpack_bytes(int mode, int cin, int cout, int k);
size_t convg_wpack_bytes(int mode, int cin, int cout, int k);  // fp32 packed weights (wpack)
int launch_convg(ConvGArgs a, hipStream_t s);
int launch_convg_bf16(ConvGArgs a, hipStream_t s);
int convg_nslice(const ConvGArgs& a, int64_t* kslice);

enum MaskMode { MASK_NONE = 0, MASK_OUT = 1, MASK_BN = 2, MASK_OUT8 = 3 };
struct BwdPrepArgs {
    int B, C;
    int64_t P;
    int bps;                  // samples per slice (set by the launcher)
    const float* d;           // upstream gradient
    const float* d2;          // optional second upstream gradient (added)
    int mask_mode;            // MASK_OUT: g = d*[mask_src > 0]; MASK_BN: g = d*drop*[mask_src*s+t > 0]
    const float* mask_src;
    const uint8_t* mask8;     // MASK_OUT8: g = d*[mask8 != 0] (the block output's ReLU mask as bytes)
    const float4* mask_cf;
    const float* drop;
    float* g;                 // masked gradient (may alias d; NULL: sums only, the consumer re-masks)
    const float* y1;          // BN inputs whose sum(g*xhat) is needed (or NULL)
    const float4* cf1;
    const float* y2;
    const float4* cf2;
    float* p_g;               // [C][nslice] partial sums of g
    float* p_x1;              // [C][nslice] partial sums of g*xhat1
    float* p_x2;
    // d read from the parity-class planes of a stride-2 data gradient (ConvGArgs::par_out) instead of
    // a plain plane (no interleave pass): element (h, w) of an H x W plane lives in class
    // q = 2 (h & 1) + (w & 1) at dpar + dpo[q] ([B][C][IHc][IWc] per class, par_off)
    const float* dpar;
    int64_t dpo[4];
    int H, W;
};
int launch_bwd_prep(BwdPrepArgs a, int* nslice, hipStream_t s);
int chan_slices(int B, int C, int* bps);
int launch_chan_stats(const float* y, int B, int C, int64_t P, float* part0, float* part1, float* partn,
                      int* nslice, hipStream_t s);
int launch_bn_act(const float* y, const float4* cf, const float* res, const float4* rcf, const float* drop,
                  float* out, int B, int C, int64_t P, hipStream_t s);
int launch_bn_bwd_apply(const float* g, const float* y, const float4* cf, float* dy, int B, int C, int64_t P,
                        hipStream_t s);
int launch_maxpool3_fwd(const float* y, const float4* cf, float* out, uint8_t* arg, int B, int C, int H, int W,
                        int OH, int OW, hipStream_t s);
int launch_maxpool3_bwd(const uint8_t* arg, const float* dout, float* dz, int B, int C, int H, int W, int OH, int OW,
                        hipStream_t s);
// MaxPool(3,2,1) + ReLU backward fused with the stem BN's backward partial sums (g written once).
// The BN input comes from the y plane, or (ysel != nullptr, y unused) from the pooled plane of the
// selected taps' inputs (the fused stem, which keeps no y plane).
bool maxpool3_bwd_prep_fits(int H, int W, int OH, int OW);
// dout2 (optional): a second pooled gradient added to dout (block 0's identity-shortcut gradient)
int launch_maxpool3_bwd_prep(const uint8_t* arg, const float* dout, const float* y, const float* ysel, const float4* cf, float* g,
                             float* p_g, float* p_x, int B, int C, int H, int W, int OH, int OW, int* nslice,
                             hipStream_t s, const float* dout2 = nullptr);
int launch_fill_cf(float4* cf, int C, float4 v, hipStream_t s);

}  // namespace pcx
