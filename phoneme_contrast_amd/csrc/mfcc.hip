// On-GPU feature path of the reference's data pipeline:
//   MFCCExtractor / MelSpectrogramExtractor (src/datasets/features.py:22-150: torchaudio MFCC =
//   MelSpectrogram -> AmplitudeToDB -> DCT-II ortho, optional ComputeDeltas), the waveform gain of
//   PhonemeContrastiveDataset._augment_waveform (src/datasets/dataset.py:147-172), and the
//   spectrogram augmentations TimeMask / FrequencyMask / GaussianNoise (src/datasets/transforms.py).
//
// Kernels (one view = one clip of S samples; frames T = 1 + S / hop, center=True reflect pad):
//   melspec_kernel     block per (view, 32 frames): the reflect-padded, gained samples of the
//                      frames staged in LDS once; |DFT|^2 as a GEMM on v_mfma_f32_32x32x2_f32
//                      (A = frames x samples windowed on the fly, B = cos / sin from a 2 n_fft
//                      twiddle table indexed by (n * bin) mod n_fft); power tile in LDS; mel
//                      projection as a second MFMA GEMM against the host-built filterbank;
//                      mel [view][n_mels][T] + per-tile maxima written.
//   group_max_kernel   AmplitudeToDB's top_db floor is taken over a packed group of clips (one clip
//                      in the reference's data path, the whole batch for a batched extractor call).
//   mel_db_dct_kernel  10 log10(max(mel, 1e-10)), floor at group max - top_db, DCT-II (ortho) to
//                      n_mfcc coefficients (or log-mel output), in frame chunks staged in LDS.
//   deltas_kernel      ComputeDeltas(win_length 5, replicate padding).
//   specaug_kernel     time / frequency bands zeroed, + level * N(0,1) noise (given, or from a
//                      counter-based hash: distribution-equal, not torch-RNG-equal).
// The random draws themselves (gain, bands, noise levels) are made on the host with the
// reference's own RNG calls (phoneme_contrast_amd/transforms.py), so masks are bit-identical.
#include "pcx_common.h"

namespace pcx {
namespace {

constexpr int FT = 32;       // frames per melspec block (MFMA M)
constexpr int NGMAX = 2;     // bin groups of 32 per wave (n_fft / 2 + 1 <= 8 * 32)

struct MelArgs {
    const float* wave;
    const float* gain;   // [n] or null
    const float* fb;     // [nbp][nmp] zero-padded filterbank (host built, float32 as torchaudio)
    float* mel;          // [n][n_mels][T]
    float* tmax;         // [n][ntile]
    int64_t S;
    int n_fft, hop, n_freq, n_mels, nbg, nmp, T, ntile;
};

__device__ __forceinline__ int64_t reflect_idx(int64_t i, int64_t S) {
    if (i < 0) i = -i;
    if (i >= S) i = 2 * (S - 1) - i;
    return i;
}

__global__ __launch_bounds__(256) void melspec_kernel(MelArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int v = blockIdx.y, tile = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, l32 = lane & 31;
    const int wave = tid >> 6;
    const int span = (FT - 1) * a.hop + a.n_fft;
    const int PS = a.nbg * 32 + 1;  // power tile row stride (odd: frame-strided reads conflict-free)
    float* xs = smem;                              // [span]
    float* ct = xs + span;                         // [n_fft] cos(2 pi j / n_fft)
    float* st = ct + a.n_fft;                      // [n_fft] sin
    float* wn = st + a.n_fft;                      // [n_fft] periodic hann window
    float* P = wn + a.n_fft;                       // [FT][PS] power tile
    float* red = P + FT * PS;                      // [4] block max
    const int64_t S = a.S;
    const int f0 = tile * FT;
    const float g = a.gain ? a.gain[v] : 1.f;
    const float* wv = a.wave + (int64_t)v * S;
    const int pad = a.n_fft / 2;
    for (int j = tid; j < span; j += 256) {
        const int64_t p = (int64_t)f0 * a.hop + j - pad;  // sample index before reflection
        xs[j] = (p < S + pad) ? wv[reflect_idx(p, S)] * g : 0.f;
    }
    for (int j = tid; j < a.n_fft; j += 256) {
        double sn, cs;
        sincospi(2.0 * j / a.n_fft, &sn, &cs);
        ct[j] = (float)cs;
        st[j] = (float)sn;
        wn[j] = 0.5f - 0.5f * (float)cs;
    }
    __syncthreads();

    // |DFT|^2: D[frame][bin] = (sum_n xw[frame][n] cos)^2 + (sum_n xw sin)^2
    f32x16 ac[NGMAX], as[NGMAX];
    int idx[NGMAX], inc[NGMAX];
#pragma unroll
    for (int gi = 0; gi < NGMAX; ++gi) {
        ac[gi] = f32x16{0.f};
        as[gi] = f32x16{0.f};
        const int b = (wave + 4 * gi) * 32 + l32;
        idx[gi] = (h * b) % a.n_fft;
        inc[gi] = (2 * b) % a.n_fft;
    }
    const int ng = (a.nbg - wave + 3) / 4;  // groups of this wave (uniform)
    const float* xf = xs + l32 * a.hop;
    for (int k = 0; k < a.n_fft / 2; ++k) {  // uniform trip count: every lane takes part in every MFMA
        const int n = 2 * k + h;
        const float av = xf[n] * wn[n];
#pragma unroll
        for (int gi = 0; gi < NGMAX; ++gi) {
            if (gi < ng) {
                ac[gi] = mfma32(av, ct[idx[gi]], ac[gi]);
                as[gi] = mfma32(av, st[idx[gi]], as[gi]);
                idx[gi] += inc[gi];
                if (idx[gi] >= a.n_fft) idx[gi] -= a.n_fft;
            }
        }
    }
#pragma unroll
    for (int gi = 0; gi < NGMAX; ++gi) {
        if (gi < ng) {
            const int b = (wave + 4 * gi) * 32 + l32;
#pragma unroll
            for (int r = 0; r < 16; ++r) P[acc_row(r, h) * PS + b] = ac[gi][r] * ac[gi][r] + as[gi][r] * as[gi][r];
        }
    }
    __syncthreads();

    // mel: M[frame][m] = sum_bin P[frame][bin] fb[bin][m]
    float mx = 0.f;
    const int nmt = a.nmp / 32;
    for (int t = wave; t < nmt; t += 4) {
        f32x16 acc = f32x16{0.f};
        const float* fbt = a.fb + t * 32 + l32;
        for (int k = 0; k < a.nbg * 16; ++k) {
            const int kb = 2 * k + h;
            acc = mfma32(P[l32 * PS + kb], fbt[(int64_t)kb * a.nmp], acc);
        }
        const int m = t * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int fr = f0 + acc_row(r, h);
            if (m < a.n_mels && fr < a.T) {
                a.mel[((int64_t)v * a.n_mels + m) * a.T + fr] = acc[r];
                mx = fmaxf(mx, acc[r]);
            }
        }
    }
    mx = wave_max(mx);
    if (lane == 0) red[wave] = mx;
    __syncthreads();
    if (tid == 0) a.tmax[(int64_t)v * a.ntile + tile] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

__global__ __launch_bounds__(256) void group_max_kernel(const float* tmax, int64_t n, int ntile, int G, float* gmax) {
    __shared__ float red[4];
    const int64_t grp = blockIdx.x;
    const int64_t lo = grp * G * ntile, hi = min<int64_t>(n, (grp + 1) * G) * ntile;
    float m = 0.f;
    for (int64_t i = lo + threadIdx.x; i < hi; i += 256) m = fmaxf(m, tmax[i]);
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) gmax[grp] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

constexpr int TC = 64;  // frames per mel_db_dct chunk

// out[v][k][t] (view stride out_stride) = sum_m dct[m][k] * dB(mel[v][m][t]); dct == null: log-mel
__global__ __launch_bounds__(256) void mel_db_dct_kernel(const float* mel, const float* gmax, int G, int n_mels,
                                                         int T, const float* dct, int n_out, float top_db,
                                                         float* out, int64_t out_stride) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int v = blockIdx.x, tid = threadIdx.x;
    float* db = smem;                       // [n_mels][TC]
    float* dt = db + n_mels * TC;           // [n_mels][n_out]
    if (dct)
        for (int i = tid; i < n_mels * n_out; i += 256) dt[i] = dct[i];
    // AmplitudeToDB: 10 log10(max(x, 1e-10)) (ref 1.0), floor max_dB - top_db over the packed group
    const float floor_db = top_db > 0.f ? 10.f * log10f(fmaxf(gmax[v / G], 1e-10f)) - top_db : -INFINITY;
    const float* mv = mel + (int64_t)v * n_mels * T;
    float* ov = out + (int64_t)v * out_stride;
    for (int t0 = 0; t0 < T; t0 += TC) {
        const int tc = min(TC, T - t0);
        __syncthreads();
        for (int i = tid; i < n_mels * TC; i += 256) {
            const int m = i / TC, t = i - m * TC;
            float d = 0.f;
            if (t < tc) d = fmaxf(10.f * log10f(fmaxf(mv[(int64_t)m * T + t0 + t], 1e-10f)), floor_db);
            db[i] = d;
        }
        __syncthreads();
        if (dct) {
            for (int i = tid; i < n_out * TC; i += 256) {
                const int k = i / TC, t = i - k * TC;
                if (t >= tc) continue;
                float s = 0.f;
                for (int m = 0; m < n_mels; ++m) s = fmaf(dt[m * n_out + k], db[m * TC + t], s);
                ov[(int64_t)k * T + t0 + t] = s;
            }
        } else {
            for (int i = tid; i < n_mels * TC; i += 256) {
                const int m = i / TC, t = i - m * TC;
                if (t < tc) ov[(int64_t)m * T + t0 + t] = db[i];
            }
        }
    }
}

// torchaudio ComputeDeltas(win_length=5, mode="replicate"): (sum_k k (c[t+k] - c[t-k])) / 10
__global__ void deltas_kernel(const float* in, int64_t in_stride, float* out, int64_t out_stride, int64_t n, int F,
                              int T) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per = (int64_t)F * T;
    if (i >= n * per) return;
    const int64_t v = i / per;
    const int r = (int)(i - v * per);
    const int f = r / T, t = r - f * T;
    const float* c = in + v * in_stride + (int64_t)f * T;
    auto at = [&](int u) { return c[min(max(u, 0), T - 1)]; };
    const float d = (1.f * (at(t + 1) - at(t - 1)) + 2.f * (at(t + 2) - at(t - 2))) / 10.f;
    out[v * out_stride + (int64_t)f * T + t] = d;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// x[v][f][t] = (t in tband[v] or f in fband[v] ? 0 : x) + level[v] * noise   (Compose order:
// TimeMask, FrequencyMask, GaussianNoise, transforms.py:147-182)
__global__ void specaug_kernel(float* x, int64_t n, int F, int T, const int* tband, const int* fband,
                               const float* level, const float* noise, uint64_t seed) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per = (int64_t)F * T;
    if (i >= n * per) return;
    const int64_t v = i / per;
    const int r = (int)(i - v * per);
    const int f = r / T, t = r - f * T;
    float y = x[i];
    if (tband && t >= tband[2 * v] && t < tband[2 * v + 1]) y = 0.f;
    if (fband && f >= fband[2 * v] && f < fband[2 * v + 1]) y = 0.f;
    const float lv = level ? level[v] : 0.f;
    if (lv != 0.f) {
        float z;
        if (noise) {
            z = noise[i];
        } else {  // Box-Muller on a counter-based hash of (seed, element)
            const uint64_t u = mix64(seed ^ mix64((uint64_t)i));
            const float u1 = ((float)(u >> 40) + 1.f) * (1.f / 16777217.f);
            const float u2 = (float)((u >> 16) & 0xFFFFFF) * (1.f / 16777216.f);
            z = sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
        }
        y += lv * z;
    }
    x[i] = y;
}

}  // namespace
}  // namespace pcx

using namespace pcx;

extern "C" int pcx_melspec(const float* wave, int64_t n, int64_t S, const float* gain, const float* fb, int n_fft,
                           int hop, int n_mels, int fb_rows, int fb_cols, float* mel, float* tile_max,
                           hipStream_t stream) {
    PCX_CHECK_ARG(wave && fb && mel && tile_max, "melspec: NULL pointer");
    PCX_CHECK_ARG(n > 0 && n < 65536, "melspec: %lld clips (1..65535 per call)", (long long)n);
    PCX_CHECK_ARG(n_fft >= 2 && n_fft % 2 == 0 && hop > 0, "melspec: n_fft %d / hop %d", n_fft, hop);
    PCX_CHECK_ARG(S > n_fft / 2, "melspec: reflect padding needs more than n_fft/2 = %d samples, got %lld",
                  n_fft / 2, (long long)S);
    MelArgs a;
    a.wave = wave; a.gain = gain; a.fb = fb; a.mel = mel; a.tmax = tile_max;
    a.S = S; a.n_fft = n_fft; a.hop = hop; a.n_freq = n_fft / 2 + 1; a.n_mels = n_mels;
    a.nbg = ceil_div(a.n_freq, 32);
    a.nmp = ceil_div(n_mels, 32) * 32;
    PCX_CHECK_ARG(a.nbg <= 4 * NGMAX, "melspec: n_fft %d gives %d frequency bins (at most %d)", n_fft, a.n_freq,
                  4 * NGMAX * 32);
    PCX_CHECK_ARG(fb_rows == a.nbg * 32 && fb_cols == a.nmp, "melspec: filterbank must be zero-padded to [%d][%d]",
                  a.nbg * 32, a.nmp);
    a.T = (int)(1 + S / hop);
    a.ntile = ceil_div(a.T, FT);
    const size_t smem = ((size_t)(FT - 1) * hop + n_fft + 3 * (size_t)n_fft + (size_t)FT * (a.nbg * 32 + 1) + 4) * 4;
    PCX_CHECK_ARG(smem <= 160 * 1024, "melspec: hop %d / n_fft %d need %zu B of LDS", hop, n_fft, smem);
    (void)hipFuncSetAttribute((const void*)melspec_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    melspec_kernel<<<dim3((unsigned)a.ntile, (unsigned)n), 256, smem, stream>>>(a);
    PCX_LAUNCH_CHECK("melspec_kernel");
    return PCX_OK;
}

extern "C" int pcx_mel_finish(const float* mel, const float* tile_max, int64_t n, int64_t T, int n_mels,
                              int clamp_group, float top_db, const float* dct, int n_out, float* gmax_ws,
                              float* out, int64_t out_stride, hipStream_t stream) {
    PCX_CHECK_ARG(mel && tile_max && gmax_ws && out, "mel_finish: NULL pointer");
    PCX_CHECK_ARG(n > 0 && n < (1 << 30) && T > 0 && n_mels > 0, "mel_finish: bad sizes");
    PCX_CHECK_ARG(clamp_group >= 1, "mel_finish: clamp group %d", clamp_group);
    if (!dct) n_out = n_mels;
    PCX_CHECK_ARG(out_stride >= (int64_t)n_out * T, "mel_finish: output view stride %lld < %lld",
                  (long long)out_stride, (long long)n_out * T);
    const int ntile = ceil_div(T, FT);
    const int64_t ngroup = (n + clamp_group - 1) / clamp_group;
    group_max_kernel<<<(unsigned)ngroup, 256, 0, stream>>>(tile_max, n, ntile, clamp_group, gmax_ws);
    PCX_LAUNCH_CHECK("group_max_kernel");
    const size_t smem = ((size_t)n_mels * TC + (dct ? (size_t)n_mels * n_out : 0)) * 4;
    PCX_CHECK_ARG(smem <= 160 * 1024, "mel_finish: n_mels %d x n_mfcc %d too large", n_mels, n_out);
    (void)hipFuncSetAttribute((const void*)mel_db_dct_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)smem);
    mel_db_dct_kernel<<<(unsigned)n, 256, smem, stream>>>(mel, gmax_ws, clamp_group, n_mels, (int)T, dct, n_out,
                                                          top_db, out, out_stride);
    PCX_LAUNCH_CHECK("mel_db_dct_kernel");
    return PCX_OK;
}

extern "C" int pcx_compute_deltas(const float* in, int64_t in_stride, float* out, int64_t out_stride, int64_t n,
                                  int F, int64_t T, hipStream_t stream) {
    PCX_CHECK_ARG(in && out && n >= 0 && F > 0 && T > 0, "compute_deltas: bad arguments");
    const int64_t tot = n * F * T;
    if (!tot) return PCX_OK;
    deltas_kernel<<<ceil_div(tot, 256), 256, 0, stream>>>(in, in_stride, out, out_stride, n, F, (int)T);
    PCX_LAUNCH_CHECK("deltas_kernel");
    return PCX_OK;
}

extern "C" int pcx_specaug(float* x, int64_t n, int F, int64_t T, const int* tband, const int* fband,
                           const float* level, const float* noise, uint64_t seed, hipStream_t stream) {
    PCX_CHECK_ARG(x && n >= 0 && F > 0 && T > 0, "specaug: bad arguments");
    const int64_t tot = n * F * T;
    if (!tot) return PCX_OK;
    specaug_kernel<<<ceil_div(tot, 256), 256, 0, stream>>>(x, n, F, (int)T, tband, fband, level, noise, seed);
    PCX_LAUNCH_CHECK("specaug_kernel");
    return PCX_OK;
}
