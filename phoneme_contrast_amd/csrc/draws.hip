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
#include <cstdint>
#include <cstdlib>

#include "pcx_common.h"

namespace pcx {
namespace {

struct MT19937 {
    uint32_t mt[624];
    int mti = 625;

    void init_genrand(uint32_t s) {
        mt[0] = s;
        for (int i = 1; i < 624; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
        mti = 624;
    }
    void init_by_array(const uint32_t* key, int len) {  // CPython Modules/_randommodule.c
        init_genrand(19650218u);
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
        mti = 624;
    }
    uint32_t next() {
        if (mti >= 624) {
            for (int k = 0; k < 624; ++k) {
                const uint32_t y = (mt[k] & 0x80000000u) | (mt[(k + 1) % 624] & 0x7fffffffu);
                mt[k] = mt[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
            }
            mti = 0;
        }
        uint32_t y = mt[mti++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
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

struct TorchCpu {  // torch.manual_seed + torch.rand(1) (float32)
    MT19937 g;
    void seed(int64_t s) { g.init_genrand((uint32_t)((uint64_t)s & 0xffffffffu)); }
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

extern "C" int pcx_draw_view_params(const int64_t* gain_seeds, const int64_t* aug_seeds, int64_t n, int F, int T,
                                    const pcx_aug_config* cfg, float* gain, int* tband, int* fband, float* level) {
    PCX_CHECK_ARG(n >= 0 && F > 0 && T > 0, "draw_view_params: bad sizes");
    PCX_CHECK_ARG(!gain_seeds || gain, "draw_view_params: gain seeds without gain output");
    PCX_CHECK_ARG(!aug_seeds || (cfg && tband && fband && level), "draw_view_params: NULL output");
    PyRandom py;
    TorchCpu tc;
    for (int64_t v = 0; v < n; ++v) {
        if (gain_seeds) {
            py.seed(gain_seeds[v]);
            gain[v] = py.random() < 0.5 ? (float)py.uniform(0.8, 1.2) : 1.0f;
        }
        if (!aug_seeds) continue;
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
    return PCX_OK;
}
