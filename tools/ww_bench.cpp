// Standalone timing + cross-check of the Winograd weight gradient (wgrad_wino) against the
// pixel-stream kernel (wgrad_s) on one layer shape (analysis aid; tests/test_wino_engine_gpu.py
// runs it on the cnn_small shapes).
//   ww_bench H W cin cout [B] [reps] [pro]
// Prints both times, dW relative difference (max |a - b| / max |b|) and the dy difference.
#include <algorithm>
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
template <class A, class F>
static float timeit(F f, int pro, A a, int reps) {
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    if (f(pro, a, 0)) {
        char msg[512];
        pcx_last_error(msg, sizeof msg);
        printf("launch failed: %s\n", msg);
        exit(1);
    }
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) f(pro, a, 0);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}
// dz[b][c][2h + i][2w + j] = sel[b][c][h][w] == 2 i + j ? dp[b][c][h][w] : 0  (pd mode: the reference's dz)
__global__ void expand_pool(const float* dp, const uint8_t* sel, float* dz, size_t np, int Wp) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i < np; i += (size_t)gridDim.x * blockDim.x) {
        const size_t row = i / Wp, w = i - row * Wp;
        const int s = sel[i] & 3;
        float* o = dz + (2 * row) * (2 * (size_t)Wp) + 2 * w;
        o[0] = s == 0 ? dp[i] : 0.f;
        o[1] = s == 1 ? dp[i] : 0.f;
        o[2 * Wp] = s == 2 ? dp[i] : 0.f;
        o[2 * Wp + 1] = s == 3 ? dp[i] : 0.f;
    }
}
__global__ void fill_sel(uint8_t* p, size_t n, unsigned seed) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2246822519u ^ seed;
        h ^= h >> 15; h *= 0x2c1b3c6d; h ^= h >> 12;
        p[i] = (uint8_t)(h & 3);
    }
}

int main(int argc, char** argv) {
    if (argc < 5) { printf("usage: ww_bench H W cin cout [B] [reps] [pro] [pd]\n"); return 2; }
    const bool pd = argc > 8 && atoi(argv[8]) != 0;  // wgrad_wino reads dz as a pooled gradient + selection
    int H = atoi(argv[1]), W = atoi(argv[2]), cin = atoi(argv[3]), cout = atoi(argv[4]);
    int B = argc > 5 ? atoi(argv[5]) : 4096, reps = argc > 6 ? atoi(argv[6]) : 5, pro = argc > 7 ? atoi(argv[7]) : 1;
    size_t ny = (size_t)B * cout * H * W, nx = (size_t)B * cin * H * W, nw = (size_t)cout * cin * 9;
    float *dz, *y, *x, *dy1, *dy2, *part, *cfd, *cfx, *g1, *g2;
    (void)hipMalloc(&dz, ny * 4); (void)hipMalloc(&y, ny * 4); (void)hipMalloc(&dy1, ny * 4); (void)hipMalloc(&dy2, ny * 4);
    (void)hipMalloc(&x, nx * 4); (void)hipMalloc(&cfd, cout * 16); (void)hipMalloc(&cfx, cin * 16);
    (void)hipMalloc(&g1, nw * 4); (void)hipMalloc(&g2, nw * 4);
    fill<<<4096, 256>>>(dz, ny, 1, 2.f, 0.f); fill<<<4096, 256>>>(y, ny, 2, 2.f, 0.f); fill<<<4096, 256>>>(x, nx, 3, 2.f, 0.f);
    float* dpool = nullptr;
    uint8_t* sel = nullptr;
    if (pd) {
        const size_t np = ny / 4;
        (void)hipMalloc(&dpool, np * 4); (void)hipMalloc(&sel, np);
        fill<<<4096, 256>>>(dpool, np, 9, 2.f, 0.f);
        fill_sel<<<4096, 256>>>(sel, np, 10);
        expand_pool<<<4096, 256>>>(dpool, sel, dz, np, W / 2);
    }
    fill<<<1, 256>>>(cfd, cout * 4, 4, 0.5f, 1.f); fill<<<1, 256>>>(cfx, cin * 4, 5, 0.5f, 0.5f);
    (void)hipMemset(dy1, 0, ny * 4); (void)hipMemset(dy2, 0, ny * 4);
    pcx::WgradArgs s{};
    pcx::WinoWgradArgs w{};
    // reference: the pixel-stream kernel, or at narrow widths the 32 x 32 row-window kernel
    const bool w32 = !pcx::wgrad_s_geometry(B, H, W, cin, cout, &s);
    if (w32 && !pcx::wgrad_w32_geometry(B, H, W, cin, cout, &s)) { printf("no reference geometry\n"); return 1; }
    if (!pcx::wgrad_wino_geometry(B, H, W, cin, cout, &w)) { printf("no wgrad_wino geometry\n"); return 1; }
    size_t np = std::max((size_t)s.nslice * nw, (size_t)w.nslice * cout * cin * 16);
    (void)hipMalloc(&part, np * 4);
    s.B = B; s.H = H; s.W = W; s.cin = cin; s.cout = cout;
    s.dz = dz; s.y = y; s.cf_dy = (const float4*)cfd; s.src = x; s.cf_x = (const float4*)cfx;
    s.srcH = H; s.srcW = W; s.part = part; s.dy_out = dy1;
    w.B = B; w.H = H; w.W = W; w.cin = cin; w.cout = cout;
    w.dz = pd ? nullptr : dz; w.dzpool = dpool; w.parg = sel; w.y = y; w.cf_dy = (const float4*)cfd; w.src = x; w.cf_x = (const float4*)cfx;
    w.part = part; w.dy_out = dy2;
    float ms_s = timeit<pcx::WgradArgs>(w32 ? pcx::launch_wgrad_w32 : pcx::launch_wgrad_s, pro, s, reps);
    (w32 ? pcx::launch_wgrad_w32 : pcx::launch_wgrad_s)(pro, s, 0); pcx::launch_sum_slices(part, s.nslice, nw, g1, 0);
    float ms_w = timeit<pcx::WinoWgradArgs>(pcx::launch_wgrad_wino, pro, w, reps);
    pcx::launch_wgrad_wino(pro, w, 0); pcx::launch_wgrad_wino_reduce(part, w.nslice, cout, cin, g2, 0);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) pcx::launch_wgrad_wino_reduce(part, w.nslice, cout, cin, g2, 0);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms_r; (void)hipEventElapsedTime(&ms_r, e0, e1);
    ms_r /= reps;
    if (hipDeviceSynchronize() != hipSuccess) { printf("device error\n"); return 1; }
    std::vector<float> h1(nw), h2(nw), d1(ny), d2(ny);
    (void)hipMemcpy(h1.data(), g1, nw * 4, hipMemcpyDeviceToHost); (void)hipMemcpy(h2.data(), g2, nw * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(d1.data(), dy1, ny * 4, hipMemcpyDeviceToHost); (void)hipMemcpy(d2.data(), dy2, ny * 4, hipMemcpyDeviceToHost);
    double emax = 0, gmax = 0, dmax = 0, dyabs = 0;
    int worst = 0;
    for (size_t i = 0; i < nw; ++i) {
        const double e = std::fabs((double)h1[i] - h2[i]);
        if (e > emax) { emax = e; worst = (int)i; }
        gmax = std::max(gmax, (double)std::fabs(h1[i]));
    }
    for (size_t i = 0; i < ny; ++i) { dmax = std::max(dmax, (double)std::fabs(d1[i] - d2[i])); dyabs = std::max(dyabs, (double)std::fabs(d1[i])); }
    const double fl = 2.0 * B * H * W * cin * cout * 9;
    printf("%sH%d W%d %d->%d pro%d B%d | reference: %.3f ms (%.3f of 157.3 TF) | wino S %d V %d slices %d: %.3f ms (%.3f alg, "
           "%.3f exec) + reduce %.3f ms | dW rel %.2e (worst [%d] %g vs %g) dy diff %.2e of %.2e\n",
           pd ? "(pooled dz) " : "", H, W, cin, cout, pro, B, ms_s, fl / ms_s / 1e9 / 157.3, w.S, w.V, w.nslice, ms_w, fl / ms_w / 1e9 / 157.3,
           fl * 4 / 9 / ms_w / 1e9 / 157.3, ms_r, emax / gmax, worst, h2[worst], h1[worst], dmax, dyabs);
    const bool ok = emax / gmax < 1e-4 && dmax <= 1e-6 * dyabs;
    if (!ok) {  // the first dy mismatches as (sample, channel, row, column)
        int shown = 0;
        for (size_t i = 0; i < ny && shown < 8; ++i)
            if (std::fabs((double)d1[i] - d2[i]) > 1e-6 * dyabs) {
                const size_t wq = i % W, hq = (i / W) % H, cq = (i / ((size_t)W * H)) % cout, bq = i / ((size_t)W * H * cout);
                printf("  dy mismatch b %zu c %zu h %zu w %zu: %g vs %g\n", bq, cq, hq, wq, d2[i], d1[i]);
                ++shown;
            }
    }
    return ok ? 0 : 3;
}
