// Host-side network plan shared by the cnn_small (net.hip) and cnn_deep (deep.hip) orchestrators.
#pragma once
#include <dlfcn.h>

#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "kernels.h"

namespace pcx {

struct Region {
    std::string name;
    size_t off, bytes;
};

// Optional per-launch HIP-event timing (pcx_net_profile): lets bench.py time individual kernels
// on the stream they run on, inside its timed region.
struct Profiler {
    bool on = false;
    std::string only;  // record this label alone (empty: every label)
    std::vector<hipEvent_t> pool;
    size_t used = 0;
    std::vector<std::string> labels;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> spans;
    hipEvent_t get() {
        if (used == pool.size()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) return nullptr;
            pool.push_back(e);
        }
        return pool[used++];
    }
    void clear() {
        used = 0;
        labels.clear();
        spans.clear();
    }
    ~Profiler() {
        for (auto e : pool) (void)hipEventDestroy(e);
    }
};

// Optional ROCTx ranges named like the profiler labels (env PCX_ROCTX=1): under
// `rocprofv3 --kernel-trace --marker-trace --kernel-rename` every dispatch of a labelled launch
// carries its label, which scripts/pmc_summary.py uses to key the --pmc passes of the same command
// by dispatch order.  The library is dlopen'ed, so libpcx has no profiler dependency.
struct Roctx {
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
    static Roctx& get() {
        static Roctx r = [] {
            Roctx x;
            const char* e = std::getenv("PCX_ROCTX");
            if (!e || std::strcmp(e, "1") != 0) return x;
            void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
            if (!h) h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_GLOBAL);
            if (!h) return x;
            x.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
            x.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
            if (!x.push || !x.pop) x.push = nullptr, x.pop = nullptr;
            return x;
        }();
        return r;
    }
};

struct Scope {
    Profiler* p;
    hipStream_t s;
    hipEvent_t a = nullptr;
    std::string label;
    bool tx = false;
    Scope(Profiler* prof, hipStream_t st, const char* lab, int layer = -1) : p(prof), s(st) {
        const Roctx& r = Roctx::get();
        if (!p->on && !r.push) return;
        label = lab;
        if (layer >= 0) label += "_L" + std::to_string(layer);
        if (r.push) {
            r.push(label.c_str());
            tx = true;
        }
        if (!p->on || (!p->only.empty() && label != p->only)) return;
        a = p->get();
        if (a) (void)hipEventRecord(a, s);
    }
    ~Scope() {
        if (tx) Roctx::get().pop();
        if (!a) return;
        hipEvent_t b = p->get();
        if (!b) return;
        (void)hipEventRecord(b, s);
        p->labels.push_back(label);
        p->spans.push_back({a, b});
    }
};

// Gradient buckets (pcx_net_grad_buckets): events recorded during the backward once every
// gradient of a bucket is written, so a DDP all-reduce can start behind the remaining layers.
struct GradBuckets {
    std::vector<int> first;          // descending parameter indices: bucket k = [first[k], first[k-1])
    std::vector<hipEvent_t> ev;
    std::vector<char> fired;
    void clear() {
        for (auto e : ev) (void)hipEventDestroy(e);
        ev.clear();
        first.clear();
        fired.clear();
    }
    void begin() { fired.assign(first.size(), 0); }
    // every parameter with index >= low has its final gradient on stream s
    void mark(int low, hipStream_t s) {
        for (size_t k = 0; k < first.size(); ++k)
            if (!fired[k] && first[k] >= low) {
                (void)hipEventRecord(ev[k], s);
                fired[k] = 1;
            }
    }
    ~GradBuckets() { clear(); }
};

struct Layer {  // one 3x3 conv of the trunk (L = 1..6)
    int cin, cout, H, W;   // conv resolution
    int srcH, srcW;        // resolution of the tensor its prologue reads
    bool pooled_in;        // prologue includes MaxPool2 + Dropout2d
    int drop_idx;          // dropout layer feeding its input (pooled_in) or -1
    size_t y, dz, cf, cfb, wu, wud;  // workspace offsets (wu / wud: Winograd weights, forward / data gradient)
    size_t xp;             // pooled_in: materialised input drop * maxpool2(relu(bn(y_prev)))
    size_t ysel, parg;     // pooled_in + wino: each window's selected y_prev (f32) and its index (u8), recorded
                           // by the forward's pool for the data gradient's EPI_BWD_POOLSEL epilogue
    int nblk;              // forward statistics tiles
    bool wino;             // Winograd conv (W >= 31); else the direct LDS-DMA conv (wu / wud then hold
                           // the [9][cin][cout] / flipped [9][cout][cin] packings)
    WgradArgs wg;          // weight-gradient geometry (pixel-stream kernel)
    bool wgw;              // weight gradient on the Winograd kernel (wgrad_wino.hip) instead
    WinoWgradArgs ww;
    bool wgbd;             // weight AND data gradient in one kernel (wgbd_wino.hip: layer 2, W % 4 == 0)
    WinoBwdArgs wb;
    bool pd;               // wgbd: dz read as layer 3's pooled gradient + window selection (EPI_BWD_POOLSELP)
    bool psel;             // pooled_in: ysel / parg written by the producer conv's epilogue (conv_wino POOL), xp
                           // then one light pass over ysel (pool_act) instead of bn_relu_pool (round 6)
};

struct DeepPlan;  // deep.hip

struct Plan {
    pcx_net_config cfg;
    std::shared_ptr<DeepPlan> deep;  // cnn_deep layout (null for cnn_small)
    int B, F, T, D, C6, P6;
    Layer L[7];
    int conv1_nblk, conv1_rows;
    int wg1_nslice, wg1_rows;
    size_t stat_part, stat_bytes;   // shared scratch for BN partials
    size_t wq;                      // conv_wino unit queue (0: static unit order); zeroed by each pass
    size_t dyb;                     // dy of the layer being back-propagated (DMA path)
    size_t wg_part, wg_bytes;       // shared scratch for weight-gradient partials
    size_t proj_part;
    size_t pooled, att, h, cfp, cfpb, norm, dzp, dh, dpooled, wt, hp_dz, hp_dzx, hp_dwa, hp_dba;
    size_t total;
    std::vector<Region> regions;
    int nparams, nbn, ndrop, drop_ch[4];
    mutable Profiler prof;
    mutable GradBuckets buckets;
    std::vector<int> stages;        // parameter indices at which the backward completes a stage

    size_t carve(const char* name, size_t bytes) {
        size_t off = total;
        total += (bytes + 256 + 255) / 256 * 256;  // >= 256 B slack: 16-byte conv copies may overrun a tensor end by 12 B
        regions.push_back({name, off, bytes});
        return off;
    }
};

inline int hip_status_ok(hipError_t e, const char* what) { return e == hipSuccess ? 0 : hip_status(e, what); }

template <class T>
T* at(void* ws, size_t off) {
    return reinterpret_cast<T*>(static_cast<char*>(ws) + off);
}


#define RC(x)                   \
    do {                        \
        int _rc = (x);          \
        if (_rc) return _rc;    \
    } while (0)

// cnn_small (net.hip)
int build_small(Plan& p);
int small_forward(const Plan& p, const float* const* P, float* const* bnstat, int64_t* const* nbt,
                  const float* x, const float* const* drop, int train, float* emb, void* ws,
                  hipStream_t s);
int small_backward(const Plan& p, const float* const* P, const float* x, const float* const* drop,
                   const float* emb, const float* demb, float* const* G, void* ws, hipStream_t s);
// cnn_deep (deep.hip)
int build_deep(Plan& p);
int deep_forward(const Plan& p, const float* const* P, float* const* bnstat, int64_t* const* nbt,
                 const float* x, const float* const* drop, int train, float* emb, void* ws,
                 hipStream_t s);
int deep_backward(const Plan& p, const float* const* P, const float* x, const float* const* drop,
                  const float* emb, const float* demb, float* const* G, void* ws, hipStream_t s);

}  // namespace pcx
