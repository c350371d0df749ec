// Host-side random draws of the reference's data augmentation, reproduced bit-exactly in C++ so a
// batch of views costs microseconds instead of one Python/torch reseeding round trip per transform.
//
// Per view the reference (src/datasets/dataset.py:77-103, transforms.py:25-144) reseeds Python's
// `random` (and torch's CPU generator) and draws:
//   gain (dataset.py:147-172):  random.seed(s); random.random() < 0.5 -> random.uniform(0.8, 1.2)
//   TimeMask / FrequencyMask:   random.seed(s); torch.manual_seed(s); random.random() < prob ->
//                               torchaudio mask_along_axis: value = torch.rand(1) * width,
//                               min_value = torch.rand(1) * (size - value), band = [long(min_value),
//                               long(min_value) + long(value))
//   GaussianNoise:              random.seed(s); random.random() < prob -> random.uniform(lo, hi)
// Python's random: MT19937 seeded by init_by_array(32-bit words of |s|), random() = 53-bit from
// two outputs.  torch's CPU generator: MT19937 init_genrand(s & 0xffffffff); torch.rand(1) for
// float32 = (next32 & 0xffffff) * 2^-24.  tests/test_draws_host.py checks both against Python and
// torch directly.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <thread>
#include <vector>

#include "pcx_common.h"

namespace pcx {
namespace {

// MT19937 that only ever produces the first few outputs after a reseed (each draw here needs at
// most 4): outputs k < 227 of the first twist depend only on pre-twist words k, k + 1, k + 397, so
// they are twisted on demand instead of regenerating all 624 words.
struct MT19937 {
    uint32_t mt[624];
    int next_k = 0;

    static uint32_t temper(uint32_t y) {
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        return y ^ (y >> 18);
    }
    // init_genrand(s), but only words [0, n) are formed (n = 402 suffices for 4 outputs)
    void init_genrand(uint32_t s, int n = 624) {
        mt[0] = s;
        for (int i = 1; i < n; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
        next_k = 0;
    }
    void init_by_array(const uint32_t* key, int len) {  // CPython Modules/_randommodule.c
        static const MT19937 base = [] {
            MT19937 b;
            b.init_genrand(19650218u);
            return b;
        }();
        memcpy(mt, base.mt, sizeof(mt));
        int i = 1, j = 0;
        for (int k = (624 > len ? 624 : len); k; --k) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key[j] + (uint32_t)j;
            ++i;
            ++j;
            if (i >= 624) { mt[0] = mt[623]; i = 1; }
            if (j >= len) j = 0;
        }
        for (int k = 623; k; --k) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
            ++i;
            if (i >= 624) { mt[0] = mt[623]; i = 1; }
        }
        mt[0] = 0x80000000u;
        next_k = 0;
    }
    uint32_t next() {  // output next_k of the first twist (next_k < 227)
        const int k = next_k++;
        const uint32_t y = (mt[k] & 0x80000000u) | (mt[k + 1] & 0x7fffffffu);
        return temper(mt[k + 397] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u));
    }
};

struct PyRandom {  // Python's random.Random
    MT19937 g;
    void seed(int64_t s) {
        uint64_t n = s < 0 ? (uint64_t)(-(s + 1)) + 1 : (uint64_t)s;
        uint32_t key[2] = {(uint32_t)n, (uint32_t)(n >> 32)};
        g.init_by_array(key, key[1] ? 2 : 1);
    }
    double random() {
        const uint32_t a = g.next() >> 5, b = g.next() >> 6;
        return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
    }
    double uniform(double lo, double hi) { return lo + (hi - lo) * random(); }
};

struct TorchCpu {  // torch.manual_seed + torch.rand(1) (float32); at most 2 draws per seed here
    MT19937 g;
    void seed(int64_t s) { g.init_genrand((uint32_t)((uint64_t)s & 0xffffffffu), 402); }
    float rand() { return (float)(g.next() & 0xffffffu) * (1.0f / 16777216.0f); }
};

// torchaudio mask_along_axis draw; returns false for an empty mask parameter
bool band(TorchCpu& t, int size, int width, int* out) {
    if (width < 1) return false;
    const float value = t.rand() * (float)width;
    const float min_value = t.rand() * ((float)size - value);
    const int64_t lo = (int64_t)min_value;
    out[0] = (int)lo;
    out[1] = (int)(lo + (int64_t)value);
    return true;
}

}  // namespace
}  // namespace pcx

using namespace pcx;

namespace {
constexpr int LANES = 8;

// Python random.seed for LANES seeds < 2^32 at once (identical one-word keys): the init_by_array
// recurrences of different seeds are independent, so the lane-minor layout vectorises.
struct PyBatch {
    uint32_t mt[624][LANES];
    int next_k[LANES];
    void seed(const uint32_t* key) {
        static const MT19937 base = [] {
            MT19937 b;
            b.init_genrand(19650218u);
            return b;
        }();
        for (int i = 0; i < 624; ++i)
            for (int l = 0; l < LANES; ++l) mt[i][l] = base.mt[i];
        int i = 1;
        for (int k = 624; k; --k) {  // j is always 0 for a one-word key
            for (int l = 0; l < LANES; ++l)
                mt[i][l] = (mt[i][l] ^ ((mt[i - 1][l] ^ (mt[i - 1][l] >> 30)) * 1664525u)) + key[l];
            ++i;
            if (i >= 624) {
                for (int l = 0; l < LANES; ++l) mt[0][l] = mt[623][l];
                i = 1;
            }
        }
        for (int k = 623; k; --k) {
            for (int l = 0; l < LANES; ++l)
                mt[i][l] = (mt[i][l] ^ ((mt[i - 1][l] ^ (mt[i - 1][l] >> 30)) * 1566083941u)) - (uint32_t)i;
            ++i;
            if (i >= 624) {
                for (int l = 0; l < LANES; ++l) mt[0][l] = mt[623][l];
                i = 1;
            }
        }
        for (int l = 0; l < LANES; ++l) {
            mt[0][l] = 0x80000000u;
            next_k[l] = 0;
        }
    }
    uint32_t next(int l) {
        const int k = next_k[l]++;
        const uint32_t y = (mt[k][l] & 0x80000000u) | (mt[k + 1][l] & 0x7fffffffu);
        return MT19937::temper(mt[k + 397][l] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u));
    }
    double random(int l) {
        const uint32_t a = next(l) >> 5, b = next(l) >> 6;
        return (a * 67108864.0 + b) * (1.0 / 9007199254740992.0);
    }
    double uniform(int l, double lo, double hi) { return lo + (hi - lo) * random(l); }
};

struct TorchBatch {  // torch.manual_seed for LANES seeds, words [0, 402)
    uint32_t mt[402][LANES];
    int next_k[LANES];
    void seed(const uint32_t* s) {
        for (int l = 0; l < LANES; ++l) {
            mt[0][l] = s[l];
            next_k[l] = 0;
        }
        for (int i = 1; i < 402; ++i)
            for (int l = 0; l < LANES; ++l) mt[i][l] = 1812433253u * (mt[i - 1][l] ^ (mt[i - 1][l] >> 30)) + (uint32_t)i;
    }
    float rand(int l) {
        const int k = next_k[l]++;
        const uint32_t y = (mt[k][l] & 0x80000000u) | (mt[k + 1][l] & 0x7fffffffu);
        const uint32_t o = MT19937::temper(mt[k + 397][l] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u));
        return (float)(o & 0xffffffu) * (1.0f / 16777216.0f);
    }
};

bool band_b(TorchBatch& t, int l, int size, int width, int* out) {
    if (width < 1) return false;
    const float value = t.rand(l) * (float)width;
    const float min_value = t.rand(l) * ((float)size - value);
    const int64_t lo = (int64_t)min_value;
    out[0] = (int)lo;
    out[1] = (int)(lo + (int64_t)value);
    return true;
}

// scalar path: any seed outside [0, 2^32) (two-word Python key) in a group
void draw_one(const int64_t* gain_seeds, const int64_t* aug_seeds, int64_t v, int F, int T, const pcx_aug_config* cfg,
              float* gain, int* tband, int* fband, float* level) {
    PyRandom py;
    TorchCpu tc;
    if (gain_seeds) {
        py.seed(gain_seeds[v]);
        gain[v] = py.random() < 0.5 ? (float)py.uniform(0.8, 1.2) : 1.0f;
    }
    if (!aug_seeds) return;
    tband[2 * v] = tband[2 * v + 1] = 0;
    fband[2 * v] = fband[2 * v + 1] = 0;
    level[v] = 0.f;
    int i = 0;  // index among the enabled transforms (seed + 1000 i, transforms.py:139-143)
    if (cfg->time_enabled) {
        const int64_t s = aug_seeds[v] + 1000 * (int64_t)i++;
        py.seed(s);
        tc.seed(s);
        if (py.random() < cfg->time_prob) band(tc, T, cfg->time_width, tband + 2 * v);
    }
    if (cfg->freq_enabled) {
        const int64_t s = aug_seeds[v] + 1000 * (int64_t)i++;
        py.seed(s);
        tc.seed(s);
        if (py.random() < cfg->freq_prob) band(tc, F, cfg->freq_width, fband + 2 * v);
    }
    if (cfg->noise_enabled) {
        const int64_t s = aug_seeds[v] + 1000 * (int64_t)i++;
        py.seed(s);
        if (py.random() < cfg->noise_prob) level[v] = (float)py.uniform(cfg->noise_min, cfg->noise_max);
    }
}

bool small(int64_t s) { return s >= 0 && s < ((int64_t)1 << 32); }

void draw_range(const int64_t* gain_seeds, const int64_t* aug_seeds, int64_t v0, int64_t v1, int F, int T,
                const pcx_aug_config* cfg, float* gain, int* tband, int* fband, float* level) {
    PyBatch* py = new PyBatch;
    TorchBatch* tc = new TorchBatch;
    uint32_t key[LANES];
    for (int64_t g0 = v0; g0 < v1; g0 += LANES) {
        const int m = (int)std::min<int64_t>(LANES, v1 - g0);
        bool ok = m == LANES;
        for (int l = 0; l < m && ok; ++l) {
            if (gain_seeds && !small(gain_seeds[g0 + l])) ok = false;
            if (aug_seeds && !(small(aug_seeds[g0 + l]) && small(aug_seeds[g0 + l] + 3000))) ok = false;
        }
        if (!ok) {
            for (int l = 0; l < m; ++l) draw_one(gain_seeds, aug_seeds, g0 + l, F, T, cfg, gain, tband, fband, level);
            continue;
        }
        if (gain_seeds) {
            for (int l = 0; l < LANES; ++l) key[l] = (uint32_t)gain_seeds[g0 + l];
            py->seed(key);
            for (int l = 0; l < LANES; ++l) gain[g0 + l] = py->random(l) < 0.5 ? (float)py->uniform(l, 0.8, 1.2) : 1.0f;
        }
        if (!aug_seeds) continue;
        for (int l = 0; l < LANES; ++l) {
            const int64_t v = g0 + l;
            tband[2 * v] = tband[2 * v + 1] = 0;
            fband[2 * v] = fband[2 * v + 1] = 0;
            level[v] = 0.f;
        }
        int i = 0;
        for (int kind = 0; kind < 3; ++kind) {
            const int en = kind == 0 ? cfg->time_enabled : kind == 1 ? cfg->freq_enabled : cfg->noise_enabled;
            if (!en) continue;
            for (int l = 0; l < LANES; ++l) key[l] = (uint32_t)(aug_seeds[g0 + l] + 1000 * (int64_t)i);
            ++i;
            py->seed(key);
            if (kind < 2) tc->seed(key);
            for (int l = 0; l < LANES; ++l) {
                const int64_t v = g0 + l;
                const double u = py->random(l);
                if (kind == 0 && u < cfg->time_prob) band_b(*tc, l, T, cfg->time_width, tband + 2 * v);
                if (kind == 1 && u < cfg->freq_prob) band_b(*tc, l, F, cfg->freq_width, fband + 2 * v);
                if (kind == 2 && u < cfg->noise_prob) level[v] = (float)py->uniform(l, cfg->noise_min, cfg->noise_max);
            }
        }
    }
    delete py;
    delete tc;
}
}  // namespace

extern "C" int pcx_draw_view_params(const int64_t* gain_seeds, const int64_t* aug_seeds, int64_t n, int F, int T,
                                    const pcx_aug_config* cfg, float* gain, int* tband, int* fband, float* level) {
    PCX_CHECK_ARG(n >= 0 && F > 0 && T > 0, "draw_view_params: bad sizes");
    PCX_CHECK_ARG(!gain_seeds || gain, "draw_view_params: gain seeds without gain output");
    PCX_CHECK_ARG(!aug_seeds || (cfg && tband && fband && level), "draw_view_params: NULL output");
    // each view reseeds its own generators, so views split over threads with identical results
    // (every MT19937 reseed costs ~2k steps: 4 per view)
    // (at most 16 threads: a GPU box's share of its host; the draws do not depend on the split)
    const unsigned nt0 = std::thread::hardware_concurrency();
    unsigned nt = nt0 ? nt0 : 1;
    nt = (unsigned)std::max<int64_t>(1, std::min<int64_t>({(int64_t)nt, 16, n / 256}));
    if (nt <= 1) {
        draw_range(gain_seeds, aug_seeds, 0, n, F, T, cfg, gain, tband, fband, level);
        return PCX_OK;
    }
    std::vector<std::thread> pool;
    for (unsigned t = 0; t < nt; ++t) {
        const int64_t v0 = n * t / nt, v1 = n * (t + 1) / nt;
        pool.emplace_back(draw_range, gain_seeds, aug_seeds, v0, v1, F, T, cfg, gain, tband, fband, level);
    }
    for (auto& th : pool) th.join();
    return PCX_OK;
}
