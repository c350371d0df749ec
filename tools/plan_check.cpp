// Host-side check of the plan builders (net.hip / deep.hip and the geometry / cost models they call)
// under AddressSanitizer + UndefinedBehaviorSanitizer, no GPU: `make asan` compiles every source
// host-only with the sanitizers and links this driver (tests/test_plan_asan.py runs it).
// For a grid of cnn_small / cnn_deep configurations it builds the plan, reads its workspace size, its
// parameter / BN / dropout counts and gradient stages, checks every named cnn_small region lies inside
// the workspace behind the 256-byte guard, and destroys it.  Exit 0 when every plan builds and checks.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "pcx.h"

static int fails = 0;

static void check_plan(const pcx_net_config& c, long B, long T, const char* what) {
    void* p = pcx_net_create(&c, B, 40, T);
    if (!p) {
        char msg[512];
        pcx_last_error(msg, sizeof msg);
        // a refused shape must say why (and is not a failure of the planner)
        printf("refused %s B=%ld T=%ld: %s\n", what, B, T, msg);
        if (!msg[0]) ++fails;
        return;
    }
    const size_t ws = pcx_net_workspace_bytes(p);
    int np = 0, nbn = 0, nd = 0, dch[8] = {0};
    if (pcx_net_info(p, &np, &nbn, &nd, dch) != 0 || np <= 0 || ws == 0) {
        printf("FAIL info %s B=%ld T=%ld\n", what, B, T);
        ++fails;
    }
    std::vector<int> st(64);
    const int ns = pcx_net_grad_stages(p, st.data(), (int)st.size());
    if (ns <= 0) {
        printf("FAIL stages %s B=%ld T=%ld\n", what, B, T);
        ++fails;
    }
    if (c.kind == 0) {
        const char* fam[] = {"y", "dz", "cf", "cfb", "xp", "ysel", "parg"};
        for (const char* f : fam)
            for (int l = 1; l <= 6; ++l) {
                const std::string nm = std::string(f) + std::to_string(l);
                size_t off = 0, bytes = 0;
                if (pcx_net_region(p, nm.c_str(), &off, &bytes) != 0) continue;
                if (off < 256 || off + bytes > ws) {
                    printf("FAIL region %s [%zu, +%zu) outside [256, %zu) in %s B=%ld T=%ld\n", nm.c_str(), off, bytes,
                           ws, what, B, T);
                    ++fails;
                }
            }
    }
    pcx_net_destroy(p);
}

int main() {
    const long Ts[] = {16, 31, 50, 57, 100, 101, 200, 201, 203, 256};
    const long Bs[] = {1, 3, 8, 24, 512, 4096, 32768};
    int n = 0;
    for (int att = 0; att < 2; ++att)
        for (int D : {64, 128, 256})
            for (long T : Ts)
                for (long B : Bs) {
                    pcx_net_config c{};
                    c.kind = 0;
                    c.in_channels = 1;
                    c.embedding_dim = D;
                    c.use_attention = att;
                    check_plan(c, B, T, "cnn_small");
                    ++n;
                }
    const int widths[][4] = {{64, 128, 256, 512}, {32, 64, 128, 256}, {16, 32, 64, 128}, {8, 16, 24, 40}};
    for (const auto& w : widths)
        for (int res = 0; res < 2; ++res)
            for (int bf = 0; bf < 2; ++bf)
                for (long T : {57L, 100L, 200L, 201L})
                    for (long B : {1L, 5L, 24L, 4096L}) {
                        pcx_net_config c{};
                        c.kind = 1;
                        c.in_channels = 1;
                        c.embedding_dim = 128;
                        c.use_attention = 1;
                        std::memcpy(c.hidden_dims, w, sizeof c.hidden_dims);
                        c.use_residual = res;
                        c.conv_bf16 = bf;
                        check_plan(c, B, T, "cnn_deep");
                        ++n;
                    }
    printf("plan_check: %d configurations, %d failures\n", n, fails);
    return fails ? 1 : 0;
}
