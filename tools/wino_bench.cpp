// Standalone timing + cross-check of the Winograd conv (conv_wino.hip) against the direct LDS-DMA
// conv (conv_dma.hip) on one layer shape and epilogue (analysis aid).
//   wino_bench H W cin cout [B] [reps] [epi] [pro]     epi: 0 fwd, 1 bwd relu, 2 bwd pool, 3 store,
//                                                      4 bwd pool from the recorded selection (Winograd
//                                                      EPI_BWD_POOLSEL vs the direct engine's EPI_BWD_POOL)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../phoneme_contrast_amd/csrc/kernels.h"
__global__ void fill(float* p, size_t n, unsigned seed, float scale, float off) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
        unsigned h = (unsigned)i * 2654435761u ^ seed;
        h ^= h >> 13; h *= 0x5bd1e995; h ^= h >> 15;
        p[i] = off + scale * ((h & 0xffffff) / 16777216.0f - 0.5f);
    }
}
static float timeit(int (*f)(int, int, pcx::ConvArgs, hipStream_t), int pro, int epi, pcx::ConvArgs a, int reps) {
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    if (f(pro, epi, a, 0)) { printf("launch failed\n"); exit(1); }
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) f(pro, epi, a, 0);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}
int main(int argc, char** argv) {
    if (argc < 5) { printf("usage: wino_bench H W cin cout [B] [reps] [epi] [pro]\n"); return 1; }
    int H = atoi(argv[1]), W = atoi(argv[2]), cin = atoi(argv[3]), cout = atoi(argv[4]);
    int B = argc > 5 ? atoi(argv[5]) : 4096, reps = argc > 6 ? atoi(argv[6]) : 5;
    int epi = argc > 7 ? atoi(argv[7]) : 0, pro = argc > 8 ? atoi(argv[8]) : 1;
    if (epi != 0) pro = 0;
    const bool sel = epi == 4;
    if (sel) epi = 2;  // the direct engine's epilogue; the Winograd one reads ysel / parg instead
    const int Hs = epi == 2 ? 2 * H : H, Ws = epi == 2 ? 2 * W : W;
    size_t nx = (size_t)B * cin * H * W, ny = (size_t)B * cout * Hs * Ws, nw = (size_t)cout * cin * 9;
    float *x, *xg, *w, *wp, *wu, *yp, *o1, *o2, *cfi, *cfo, *part, *drop;
    // x behind a 64-float guard of NaNs: the Winograd conv's 16-byte staging reads the float before a
    // plane (ConvArgs::src_guard) and must select it away, never multiply it in
    (void)hipMalloc(&xg, (nx + 64) * 4); x = xg + 64; (void)hipMemset(xg, 0xff, 64 * 4);
    (void)hipMalloc(&w, nw * 4); (void)hipMalloc(&wp, nw * 4);
    (void)hipMalloc(&wu, nw / 9 * 16 * 4); (void)hipMalloc(&yp, ny * 4);
    (void)hipMalloc(&o1, ny * 4); (void)hipMalloc(&o2, ny * 4);
    (void)hipMalloc(&cfi, cin * 16); (void)hipMalloc(&cfo, cout * 16); (void)hipMalloc(&drop, (size_t)B * cout * 4);
    size_t nbd = pcx::conv3x3_nblk(B, H, W, cout), nbw = pcx::wino_nblk(B, H, W, cin, cout);
    size_t nbm = std::max(nbd, nbw);
    (void)hipMalloc(&part, (2 * (size_t)cout * nbm + nbm) * 4 * 2);
    fill<<<4096, 256>>>(x, nx, 1, 2.f, 0.f); fill<<<4096, 256>>>(w, nw, 2, 0.2f, 0.f);
    fill<<<4096, 256>>>(yp, ny, 3, 2.f, 0.f); fill<<<1, 256>>>(cfi, cin * 4, 4, 0.5f, 0.5f);
    fill<<<1, 256>>>(cfo, cout * 4, 5, 0.5f, 0.5f); fill<<<256, 256>>>(drop, (size_t)B * cout, 6, 1.f, 1.f);
    // the data-gradient orientation is immaterial here: both engines get the same [cout][cin] weights
    pcx::launch_pack_fwd(w, wp, cout, cin, 0);
    pcx::launch_wino_pack(w, wu, cout, cin, 0, 0);
    (void)hipMemset(o1, 0, ny * 4); (void)hipMemset(o2, 0, ny * 4);
    pcx::ConvArgs a{};
    a.B = B; a.H = H; a.W = W; a.cin = cin; a.cout = cout; a.src = x; a.cf_in = (const float4*)cfi;
    a.srcH = H; a.srcW = W; a.yprev = yp; a.cf_out = (const float4*)cfo; a.drop_out = drop; a.Hs = Hs; a.Ws = Ws;
    pcx::ConvArgs d = a, q = a;
    d.wpack = wp; d.out = o1; d.nblk = (int)nbd; d.part0 = part; d.part1 = part + cout * nbd; d.partn = part + 2 * cout * nbd;
    q.wpack = wu; q.out = o2; q.nblk = (int)nbw; q.part0 = part + (2 * cout * nbm + nbm); q.src_guard = 1;
    q.part1 = q.part0 + cout * nbw; q.partn = q.part0 + 2 * cout * nbw;
    int* queue = nullptr;  // WINO_QUEUE=1: the Winograd conv takes its units from a work queue
    if (getenv("WINO_QUEUE") && atoi(getenv("WINO_QUEUE"))) {
        (void)hipMalloc(&queue, pcx::WINO_QUEUE_INTS * 4);
        (void)hipMemset(queue, 0, pcx::WINO_QUEUE_INTS * 4);
        q.queue = queue;
    }
    int qepi = epi;
    if (sel) {  // the forward's pool records each window's selected y and its index
        float *xp, *ys;
        uint8_t* pa;
        const size_t np = (size_t)B * cout * H * W;
        (void)hipMalloc(&xp, np * 4); (void)hipMalloc(&ys, np * 4); (void)hipMalloc(&pa, np);
        if (pcx::launch_bn_relu_pool(yp, (const float4*)cfo, drop, xp, B, cout, Hs, Ws, 0, ys, pa)) {
            printf("bn_relu_pool failed\n");
            return 1;
        }
        q.ysel = ys; q.parg = pa; qepi = pcx::EPI_BWD_POOLSEL;
        printf("wino EPI_BWD_POOL %.3f ms; ", timeit(pcx::launch_conv3x3_wino, pro, epi, q, reps));
    }
    float msd = timeit(pcx::launch_conv3x3_dma, pro, epi, d, reps);
    float msw = timeit(pcx::launch_conv3x3_wino, pro, qepi, q, reps);
    (void)hipMemset(o1, 0, ny * 4); (void)hipMemset(o2, 0, ny * 4);
    pcx::launch_conv3x3_dma(pro, epi, d, 0); pcx::launch_conv3x3_wino(pro, qepi, q, 0);
    (void)hipDeviceSynchronize();
    if (queue) {  // every launch must leave the queue zero
        std::vector<int> hq(pcx::WINO_QUEUE_INTS);
        (void)hipMemcpy(hq.data(), queue, hq.size() * 4, hipMemcpyDeviceToHost);
        for (int v : hq)
            if (v) { printf("queue left non-zero\n"); return 3; }
        printf("(queue) ");
    }
    std::vector<float> h1(ny), h2(ny);
    (void)hipMemcpy(h1.data(), o1, ny * 4, hipMemcpyDeviceToHost); (void)hipMemcpy(h2.data(), o2, ny * 4, hipMemcpyDeviceToHost);
    double emax = 0, gmax = 0;
    for (size_t i = 0; i < ny; ++i) { emax = std::max(emax, (double)std::fabs(h1[i] - h2[i])); gmax = std::max(gmax, (double)std::fabs(h1[i])); }
    // per-channel statistics partials, summed over blocks
    double smax = 0, sref = 0;
    if (epi != 3) {
        std::vector<float> p1(2 * cout * nbd), p2(2 * cout * nbw);
        (void)hipMemcpy(p1.data(), part, p1.size() * 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(p2.data(), q.part0, p2.size() * 4, hipMemcpyDeviceToHost);
        for (int c = 0; c < cout; ++c) {
            double s1 = 0, s2 = 0;
            for (size_t k = 0; k < nbd; ++k) s1 += p1[c * nbd + k];
            for (size_t k = 0; k < nbw; ++k) s2 += p2[c * nbw + k];
            smax = std::max(smax, std::fabs(s1 - s2));
            sref = std::max(sref, std::fabs(s1));
        }
    }
    double fl = 2.0 * B * H * W * cin * cout * 9;
    printf("H%d W%d %d->%d epi%d%s pro%d: direct %.3f ms (%.2f of fp32 roof)  wino %.3f ms (%.2f alg.)  |d out| %.2e of %.2e  |d sum0| %.2e of %.2e\n",
           H, W, cin, cout, epi, sel ? "sel" : "", pro, msd, fl / msd / 1e9 / 157.3, msw, fl / msw / 1e9 / 157.3, emax, gmax, smax, sref);
    // exit status: 2 when the outputs or the summed statistics partials disagree beyond fp32 noise
    const bool bad = emax > 1e-5 * gmax + 1e-6 || smax > 1e-4 * sref + 1e-3;
    return bad ? 2 : 0;
}
