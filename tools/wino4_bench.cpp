// Standalone timing + cross-check of the F(4x3, 3x3) Winograd conv (conv_wino4.hip) against the F(2x2, 3x3)
// conv (conv_wino.hip) on one layer shape and epilogue, same operands, both taking units from a work queue.
//   wino4_bench H W cin cout [B] [reps] [epi] [pro]   epi: 0 fwd (BN statistics), 1 bwd relu, 5 bwd pooled
//                                                      selection -> pooled routed gradient (EPI_BWD_POOLSELP)
// Exit status 2 when the outputs or the per-channel statistics sums disagree beyond float32 Winograd noise.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../phoneme_contrast_amd/csrc/kernels.h"
#include "pcx.h"

__global__ void fill(float* p, size_t n, unsigned seed, float scale, float off) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 13; h *= 0x5bd1e995; h ^= h >> 15;
        p[i] = off + scale * ((h & 0xffffff) / 16777216.0f - 0.5f);
    }
}

static float timeit(int (*f)(int, int, pcx::ConvArgs, hipStream_t), int pro, int epi, pcx::ConvArgs a, int reps) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    if (f(pro, epi, a, 0)) {
        char msg[512];
        pcx_last_error(msg, sizeof msg);
        printf("launch failed: %s\n", msg);
        exit(1);
    }
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) f(pro, epi, a, 0);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

// W4_SYNC=1: synchronise and check after every step (diagnostics: names the step that faults)
static void step(const char* what) {
    if (!getenv("W4_SYNC")) return;
    const hipError_t e = hipDeviceSynchronize();
    printf("  [%s] %s\n", what, hipGetErrorString(e));
    fflush(stdout);
    if (e != hipSuccess) exit(4);
}

int main(int argc, char** argv) {
    if (argc < 5) { printf("usage: wino4_bench H W cin cout [B] [reps] [epi] [pro]\n"); return 1; }
    const int H = atoi(argv[1]), W = atoi(argv[2]), cin = atoi(argv[3]), cout = atoi(argv[4]);
    const int B = argc > 5 ? atoi(argv[5]) : 4096, reps = argc > 6 ? atoi(argv[6]) : 5;
    const int epi = argc > 7 ? atoi(argv[7]) : 0;
    int pro = argc > 8 ? atoi(argv[8]) : 1;
    if (epi != 0) pro = 0;
    if (!pcx::wino4_geometry(B, H, W, cin, cout, nullptr)) { printf("no wino4 geometry\n"); return 1; }
    const bool pool = epi == pcx::EPI_BWD_POOLSELP;
    const int Hs = pool ? 2 * H : H, Ws = pool ? 2 * W : W;
    const size_t nx = (size_t)B * cin * H * W, ny = (size_t)B * cout * H * W, nw = (size_t)cout * cin * 9;
    const size_t nyp = (size_t)B * cout * Hs * Ws;
    float *xg, *x, *w, *wu, *w4, *yp, *o1, *o2, *cfi, *cfo, *part, *drop;
    (void)hipMalloc(&xg, (nx + 64) * 4);
    x = xg + 64;
    (void)hipMemset(xg, 0xff, 64 * 4);  // NaN guard: the 16-byte staging reads the float before a plane
    (void)hipMalloc(&w, nw * 4);
    (void)hipMalloc(&wu, (size_t)16 * cin * cout * 4);
    (void)hipMalloc(&w4, (size_t)36 * cin * cout * 4);
    (void)hipMalloc(&yp, nyp * 4);
    (void)hipMalloc(&o1, ny * 4);
    (void)hipMalloc(&o2, ny * 4);
    (void)hipMalloc(&cfi, cin * 16);
    (void)hipMalloc(&cfo, cout * 16);
    (void)hipMalloc(&drop, (size_t)B * cout * 4);
    const size_t nb2 = pcx::wino_nblk(B, H, W, cin, cout), nb4 = pcx::wino4_nblk(B, H, W, cin, cout);
    (void)hipMalloc(&part, (3 * cout * (nb2 + nb4) + 64) * 4 * 2);
    fill<<<4096, 256>>>(x, nx, 1, 2.f, 0.f);
    fill<<<4096, 256>>>(w, nw, 2, 0.2f, 0.f);
    fill<<<4096, 256>>>(yp, nyp, 3, 2.f, 0.f);
    fill<<<1, 256>>>(cfi, cin * 4, 4, 0.5f, 0.5f);
    fill<<<1, 256>>>(cfo, cout * 4, 5, 0.5f, 0.5f);
    fill<<<256, 256>>>(drop, (size_t)B * cout, 6, 1.f, 1.f);
    step("fill");
    pcx::launch_wino_pack(w, wu, cout, cin, 0, 0);
    step("wino_pack");
    pcx::launch_wino4_pack(w, w4, cout, cin, 0, 0);
    step("wino4_pack");
    int *q1, *q2;
    (void)hipMalloc(&q1, pcx::WINO_QUEUE_INTS * 4);
    (void)hipMalloc(&q2, pcx::WINO_QUEUE_INTS * 4);
    (void)hipMemset(q1, 0, pcx::WINO_QUEUE_INTS * 4);
    (void)hipMemset(q2, 0, pcx::WINO_QUEUE_INTS * 4);
    pcx::ConvArgs a{};
    a.B = B; a.H = H; a.W = W; a.cin = cin; a.cout = cout; a.src = x; a.cf_in = (const float4*)cfi;
    a.srcH = H; a.srcW = W; a.yprev = yp; a.cf_out = (const float4*)cfo; a.drop_out = drop; a.Hs = Hs; a.Ws = Ws;
    a.src_guard = 1;
    float *ys = nullptr;
    uint8_t* pa = nullptr;
    if (pool) {  // the forward's pool records each window's selected y and its index
        float* xp;
        (void)hipMalloc(&xp, ny * 4);
        (void)hipMalloc(&ys, ny * 4);
        (void)hipMalloc(&pa, ny);
        if (pcx::launch_bn_relu_pool(yp, (const float4*)cfo, drop, xp, B, cout, Hs, Ws, 0, ys, pa)) {
            printf("bn_relu_pool failed\n");
            return 1;
        }
        a.ysel = ys; a.parg = pa;
        step("bn_relu_pool");
    }
    pcx::ConvArgs q2a = a, q4a = a;
    q2a.wpack = wu; q2a.out = o1; q2a.nblk = (int)nb2; q2a.part0 = part; q2a.part1 = part + cout * nb2;
    q2a.partn = part + 2 * cout * nb2; q2a.queue = q1;
    q4a.wpack = w4; q4a.out = o2; q4a.nblk = (int)nb4; q4a.part0 = part + 3 * cout * nb2 + 32;
    q4a.part1 = q4a.part0 + cout * nb4; q4a.partn = q4a.part0 + 2 * cout * nb4; q4a.queue = q2;
    if (pool) { q2a.dpool = o1; q4a.dpool = o2; }
    const float ms2 = timeit(pcx::launch_conv3x3_wino, pro, epi, q2a, reps);
    step("conv_wino");
    const float ms4 = timeit(pcx::launch_conv3x3_wino4, pro, epi, q4a, reps);
    step("conv_wino4");
    (void)hipMemset(o1, 0, ny * 4);
    (void)hipMemset(o2, 0, ny * 4);
    if (pcx::launch_conv3x3_wino(pro, epi, q2a, 0) || pcx::launch_conv3x3_wino4(pro, epi, q4a, 0)) {
        char msg[512];
        pcx_last_error(msg, sizeof msg);
        printf("launch failed: %s\n", msg);
        return 1;
    }
    (void)hipDeviceSynchronize();
    std::vector<int> hq(pcx::WINO_QUEUE_INTS);
    (void)hipMemcpy(hq.data(), q2, hq.size() * 4, hipMemcpyDeviceToHost);
    for (int v : hq)
        if (v) { printf("queue left non-zero\n"); return 3; }
    std::vector<float> h1(ny), h2(ny);
    (void)hipMemcpy(h1.data(), o1, ny * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(h2.data(), o2, ny * 4, hipMemcpyDeviceToHost);
    double emax = 0, gmax = 0;
    size_t bad_i = 0;
    for (size_t i = 0; i < ny; ++i) {
        const double e = std::fabs((double)h1[i] - h2[i]);
        if (!(e <= emax)) { emax = e; bad_i = i; }
        gmax = std::max(gmax, (double)std::fabs(h1[i]));
    }
    std::vector<float> p2(2 * cout * nb2), p4(2 * cout * nb4);
    (void)hipMemcpy(p2.data(), part, p2.size() * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(p4.data(), q4a.part0, p4.size() * 4, hipMemcpyDeviceToHost);
    double smax = 0, sref = 0;
    for (int k = 0; k < (epi == 0 ? 1 : 2); ++k)  // forward: the sums (M2 depends on the blocking); backward: both sums
        for (int c = 0; c < cout; ++c) {
            double s2 = 0, s4 = 0;
            for (size_t b = 0; b < nb2; ++b) s2 += p2[(size_t)(k * cout + c) * nb2 + b];
            for (size_t b = 0; b < nb4; ++b) s4 += p4[(size_t)(k * cout + c) * nb4 + b];
            smax = std::max(smax, std::fabs(s2 - s4));
            sref = std::max(sref, std::fabs(s2));
        }
    const double fl = 2.0 * B * H * W * cin * cout * 9;
    printf("wino4 H%d W%d %d->%d B%d epi%d pro%d: F(2x2) %.3f ms (%.3f exec)  F(4x3) %.3f ms (%.3f exec)  speedup %.3f  "
           "|d out| %.2e of %.2e (at %zu)  |d sums| %.2e of %.2e\n",
           H, W, cin, cout, B, epi, pro, ms2, fl * 4 / 9 / ms2 / 1e9 / 157.3, ms4, fl * 30 / 108 / ms4 / 1e9 / 157.3,
           ms2 / ms4, emax, gmax, bad_i, smax, sref);
    const bool bad = !(emax <= 3e-5 * gmax + 1e-6) || !(smax <= 1e-4 * sref + 1e-3);
    return bad ? 2 : 0;
}
