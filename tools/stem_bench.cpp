// Standalone timing + cross-check of the fused bf16 stem (y0 recomputed, conv.hip stem_pool_kernel /
// stem_wgrad_rc_kernel) against the unfused kernels that keep the y0 plane (analysis aid; run by
// tools/run_stem.sh on the GPU box).
//   stem_bench [B] [H] [W] [reps]
// Checks, bit for bit: statistics-only partials vs the storing pass; a0 / taps / NHWC image vs
// maxpool3_fwd + to_nhwc on the stored y0; y0 at the selected taps vs the stored y0 (first samples,
// on the host); pooled-gradient g and the BN0 backward sums vs maxpool3_bwd_prep on y0.  The weight
// gradients differ only in summation order: relative difference printed (max |a - b| / max |b|).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
__global__ void count_diff(const unsigned char* a, const unsigned char* b, size_t n, unsigned long long* cnt) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    unsigned long long c = 0;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) c += a[i] != b[i];
    if (c) atomicAdd(cnt, c);
}
static unsigned long long ndiff(const void* a, const void* b, size_t bytes) {
    unsigned long long* d;
    (void)hipMalloc(&d, 8);
    (void)hipMemset(d, 0, 8);
    count_diff<<<4096, 256>>>((const unsigned char*)a, (const unsigned char*)b, bytes, d);
    unsigned long long h = 0;
    (void)hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return h;
}
static void check(int rc, const char* what) {
    if (rc) {
        char msg[512];
        pcx_last_error(msg, sizeof msg);
        printf("%s failed: %s\n", what, msg);
        exit(1);
    }
}
template <class F>
static float timeit(F f, int reps) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    f();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) f();
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}
static double rel(const float* d1, const float* d2, int n) {
    std::vector<float> h1(n), h2(n);
    (void)hipMemcpy(h1.data(), d1, n * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(h2.data(), d2, n * 4, hipMemcpyDeviceToHost);
    double e = 0, m = 0;
    for (int i = 0; i < n; ++i) {
        e = std::max(e, (double)std::fabs(h1[i] - h2[i]));
        m = std::max(m, (double)std::fabs(h1[i]));
    }
    return m > 0 ? e / m : e;
}

int main(int argc, char** argv) {
    const int B = argc > 1 ? atoi(argv[1]) : 4096, H = argc > 2 ? atoi(argv[2]) : 40, W = argc > 3 ? atoi(argv[3]) : 200;
    const int reps = argc > 4 ? atoi(argv[4]) : 5, C = 64;
    const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
    if (!pcx::stem_fused_ok(C, H, W)) { printf("fused stem unsupported at %dx%d\n", H, W); return 1; }
    const size_t HW = (size_t)H * W, OHW = (size_t)OH * OW, ny = (size_t)B * C * HW, np = (size_t)B * C * OHW;
    const size_t nn = (size_t)B * (OH + 2) * (OW + 2) * C;
    int rows, srows;
    const int nblk = pcx::stem_nblk(B, H, &rows);
    const int ns = pcx::stem_wgrad_nslice(B, H, &srows, true);
    const size_t npart = (size_t)3 * C * nblk + nblk;
    float *x, *w, *wr, *y0, *part1, *part2, *a1, *a2, *ysel, *dout, *g1, *g2, *pg1, *pg2, *wp, *dw1, *dw2;
    float4 *cf, *cfb;
    uint8_t *arg1, *arg2;
    void *n1, *n2;
    (void)hipMalloc(&x, (size_t)B * HW * 4); (void)hipMalloc(&w, C * 49 * 4); (void)hipMalloc(&wr, C * 49 * 4);
    (void)hipMalloc(&y0, ny * 4);
    (void)hipMalloc(&part1, npart * 4); (void)hipMalloc(&part2, npart * 4);
    (void)hipMalloc(&a1, np * 4); (void)hipMalloc(&a2, np * 4); (void)hipMalloc(&ysel, np * 4); (void)hipMalloc(&dout, np * 4);
    (void)hipMalloc(&arg1, np); (void)hipMalloc(&arg2, np);
    (void)hipMalloc(&n1, nn * 2); (void)hipMalloc(&n2, nn * 2);
    (void)hipMalloc(&g1, ny * 4); (void)hipMalloc(&g2, ny * 4);
    (void)hipMalloc(&pg1, (size_t)2 * C * B * 4); (void)hipMalloc(&pg2, (size_t)2 * C * B * 4 + 64);
    (void)hipMalloc(&wp, (size_t)ns * C * 49 * 4); (void)hipMalloc(&dw1, C * 49 * 4); (void)hipMalloc(&dw2, C * 49 * 4);
    (void)hipMalloc(&cf, C * 16); (void)hipMalloc(&cfb, C * 16);
    fill<<<4096, 256>>>(x, (size_t)B * HW, 1, 4.f, 0.f);
    fill<<<64, 256>>>(w, C * 49, 2, 0.6f, 0.f);
    fill<<<4096, 256>>>(dout, np, 3, 2.f, 0.f);
    {  // BN coefficients {scale, shift, mean, istd}: some negative scales (the pool then selects minima of y0)
        std::vector<float4> h(C), hb(C);
        for (int c = 0; c < C; ++c) {
            const float u = (float)((c * 37) % 64) / 64.f;
            h[c] = make_float4((c % 5 == 0 ? -1.f : 1.f) * (0.5f + u), 0.4f * (u - 0.5f), 0.1f * u, 0.8f + u);
            hb[c] = make_float4(0.7f + 0.5f * u, 0.01f * (u - 0.5f), 0.02f * u, 0.1f * (u - 0.3f));
        }
        (void)hipMemcpy(cf, h.data(), C * 16, hipMemcpyHostToDevice);
        (void)hipMemcpy(cfb, hb.data(), C * 16, hipMemcpyHostToDevice);
    }
    auto fwd_args = [&](float* out, float* part) {
        pcx::StemArgs a{};
        a.B = B; a.H = H; a.W = W; a.cout = C; a.x = x; a.w = w; a.out = out;
        a.nblk = nblk; a.rows_per_blk = rows;
        a.part0 = part; a.part1 = part + (size_t)C * nblk; a.partn = part + (size_t)2 * C * nblk;
        return a;
    };
    int fails = 0;
    auto report = [&](const char* what, unsigned long long d) {
        printf("  %-34s %s (%llu differing bytes)\n", what, d ? "MISMATCH" : "bitwise equal", d);
        fails += d != 0;
    };
    // ---- forward
    const float t_fwd = timeit([&] { check(pcx::launch_stem_fwd(fwd_args(y0, part1), 1, wr, 0), "stem_fwd"); }, reps);
    const float t_stat = timeit([&] { check(pcx::launch_stem_fwd(fwd_args(nullptr, part2), 1, wr, 0), "stem_fwd stats"); }, reps);
    const float t_mp = timeit([&] {
        check(pcx::launch_maxpool3_fwd(y0, cf, a1, arg1, B, C, H, W, OH, OW, 0), "maxpool3_fwd");
    }, reps);
    pcx::NhwcArgs t{};
    t.op = pcx::NHWC_COPY; t.B = B; t.C = C; t.H = OH; t.W = OW; t.src = a1; t.dst = n1;
    const float t_nhwc = timeit([&] { check(pcx::launch_to_nhwc(t, 0), "to_nhwc"); }, reps);
    pcx::StemArgs sp{};
    sp.B = B; sp.H = H; sp.W = W; sp.cout = C; sp.x = x; sp.w = wr; sp.cf = cf;
    sp.pool = a2; sp.pool_arg = arg2; sp.pool_ysel = ysel; sp.pool_nhwc = n2; sp.OH = OH; sp.OW = OW;
    const float t_pool = timeit([&] { check(pcx::launch_stem_pool(sp, 0), "stem_pool"); }, reps);
    {  // one launch after a 4 GB memset (no cache / TLB state left from the previous launch)
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        float tot = 0.f;
        for (int r = 0; r < 3; ++r) {
            (void)hipMemsetAsync(g1, r, ny * 4 < ((size_t)4 << 30) ? ny * 4 : ((size_t)4 << 30), 0);
            (void)hipEventRecord(e0);
            check(pcx::launch_stem_pool(sp, 0), "stem_pool");
            (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            tot += ms;
        }
        printf("fused pool after a memset: %.3f ms\n", tot / 3);
    }
    if (hipDeviceSynchronize() != hipSuccess) { printf("device error (forward)\n"); return 1; }
    printf("stem B%d %dx%d: fwd+store %.3f ms | stats only %.3f | maxpool %.3f + to_nhwc %.3f | fused pool %.3f ms\n",
           B, H, W, t_fwd, t_stat, t_mp, t_nhwc, t_pool);
    report("statistics partials", ndiff(part1, part2, npart * 4));
    report("NHWC bf16 image of a0", ndiff(n1, n2, nn * 2));
    {  // pooled NHWC taps / y0 at the taps vs the plane kernels (first samples on the host); a0 from them
        const int bs = std::min(B, 16);
        std::vector<float> hy((size_t)bs * C * HW), hs((size_t)bs * C * OHW), ha1((size_t)bs * C * OHW);
        std::vector<uint8_t> ha((size_t)bs * C * OHW), hr((size_t)bs * C * OHW);
        std::vector<float4> hc(C);
        (void)hipMemcpy(hy.data(), y0, hy.size() * 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(hs.data(), ysel, hs.size() * 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(ha1.data(), a1, ha1.size() * 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(ha.data(), arg2, ha.size(), hipMemcpyDeviceToHost);
        (void)hipMemcpy(hr.data(), arg1, hr.size(), hipMemcpyDeviceToHost);
        (void)hipMemcpy(hc.data(), cf, C * 16, hipMemcpyDeviceToHost);
        unsigned long long bad_t = 0, bad_y = 0, bad_a = 0, sel = 0;
        for (int b = 0; b < bs; ++b)
            for (int c = 0; c < C; ++c)
                for (int oh = 0; oh < OH; ++oh)
                    for (int ow = 0; ow < OW; ++ow) {
                        const size_t on = (((size_t)b * OH + oh) * OW + ow) * C + c;   // pooled NHWC
                        const size_t oc = ((size_t)b * C + c) * OHW + (size_t)oh * OW + ow;  // NCHW
                        bad_t += ha[on] != hr[oc];
                        const float a0 = std::fmax(std::fma(hs[on], hc[c].x, hc[c].y), 0.f);
                        bad_a += memcmp(&a0, &ha1[oc], 4) != 0;
                        if (ha[on] == 255) continue;
                        ++sel;
                        const int ih = 2 * oh - 1 + ha[on] / 3, iw = 2 * ow - 1 + ha[on] % 3;
                        const float v = hy[((size_t)b * C + c) * HW + (size_t)ih * W + iw];
                        bad_y += memcmp(&v, &hs[on], 4) != 0;
                    }
        report("taps (pooled NHWC)", bad_t);
        report("a0 = relu(BN0(y0 at the tap))", bad_a);
        printf("  %-34s %s (%llu of %llu selected windows differ)\n", "y0 at the selected taps", bad_y ? "MISMATCH" : "bitwise equal",
               bad_y, sel);
        fails += bad_y != 0;
    }
    // ---- backward: pooled gradient + BN0 sums, then the weight gradient
    int nsl1 = 0, nsl2 = 0;
    int bps;
    const int nsl = pcx::chan_slices(B, C, &bps);
    const float t_mb = timeit([&] {
        check(pcx::launch_maxpool3_bwd_prep(arg1, dout, y0, nullptr, cf, g1, pg1, pg1 + (size_t)C * nsl, B, C, H, W, OH, OW,
                                            &nsl1, 0), "maxpool3_bwd_prep");
    }, reps);
    uint16_t* g16;
    (void)hipMalloc(&g16, ny * 2);
    pcx::StemArgs sb{};
    sb.B = B; sb.H = H; sb.W = W; sb.cout = C; sb.OH = OH; sb.OW = OW; sb.cf = cf;
    sb.pool_arg = arg2; sb.pool_ysel = ysel; sb.dpool = dout; sb.dz16 = g16;
    sb.p_g = pg2; sb.p_x = pg2 + (size_t)C * B;
    const float t_mbs = timeit([&] { check(pcx::launch_stem_pool_bwd(sb, &nsl2, 0), "stem_pool_bwd"); }, reps);
    pcx::StemArgs sw{};
    sw.B = B; sw.H = H; sw.W = W; sw.cout = C; sw.x = x; sw.dz = g1; sw.y = y0; sw.cf_dy = cfb; sw.part = wp;
    sw.nblk = ns; sw.rows_per_blk = srows;
    const float t_wg = timeit([&] { check(pcx::launch_stem_wgrad(sw, 1, 0), "stem_wgrad"); }, reps);
    check(pcx::launch_sum_slices(wp, ns, (int64_t)C * 49, dw1, 0), "sum_slices");
    pcx::StemArgs sr = sw;
    sr.y = nullptr; sr.w = wr; sr.dz16 = g16;
    const float t_rc = timeit([&] { check(pcx::launch_stem_wgrad_rc(sr, 0), "stem_wgrad_rc"); }, reps);
    check(pcx::launch_sum_slices(wp, ns, (int64_t)C * 49, dw2, 0), "sum_slices");
    if (hipDeviceSynchronize() != hipSuccess) { printf("device error (backward)\n"); return 1; }
    printf("backward: maxpool_bwd_prep(y0) %.3f ms | stem_pool_bwd %.3f ms | wgrad(y0) %.3f ms | wgrad(recompute) %.3f ms\n",
           t_mb, t_mbs, t_wg, t_rc);
    {  // dz0 (bf16) == bf16(g) of the float path; BN0 sums regrouped over windows: rounding only
        std::vector<float> h1(ny);
        std::vector<uint16_t> h2(ny);
        (void)hipMemcpy(h1.data(), g1, ny * 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(h2.data(), g16, ny * 2, hipMemcpyDeviceToHost);
        unsigned long long d = 0;
        for (size_t i = 0; i < ny; ++i) {
            const uint16_t r = __builtin_bit_cast(uint16_t, (__bf16)h1[i]);
            d += r != h2[i];
        }
        report("pooled gradient dz0 (bf16)", d);
        std::vector<float> p1((size_t)2 * C * nsl), p2((size_t)2 * C * B);
        (void)hipMemcpy(p1.data(), pg1, p1.size() * 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(p2.data(), pg2, p2.size() * 4, hipMemcpyDeviceToHost);
        double rs = 0.0, mx = 0.0;
        for (int k = 0; k < 2; ++k)
            for (int c = 0; c < C; ++c) {
                double t1 = 0.0, t2 = 0.0;
                for (int q = 0; q < nsl; ++q) t1 += p1[((size_t)k * C + c) * nsl + q];
                for (int q = 0; q < B; ++q) t2 += p2[((size_t)k * C + c) * B + q];
                rs = std::max(rs, std::fabs(t1 - t2));
                mx = std::max(mx, std::fabs(t1));
            }
        rs = mx > 0 ? rs / mx : rs;
        printf("  %-34s rel %.2e (per-window regrouping)\n", "BN0 backward sums", rs);
        fails += !(rs < 1e-5);
    }
    const double r = rel(dw1, dw2, C * 49);
    printf("  %-34s rel %.2e (dz0 rounded to bf16)\n", "stem weight gradient", r);
    fails += !(r < 2e-2);
    const double fused = t_stat + t_pool + t_mbs + t_rc, unfused = t_fwd + t_mp + t_nhwc + t_mb + t_wg;
    printf("stem path: unfused %.3f ms -> fused %.3f ms\n", unfused, fused);
    return fails ? 3 : 0;
}
