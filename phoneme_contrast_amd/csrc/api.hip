// Library-wide C entry points: version and per-thread error reporting.
#include <stdarg.h>

#include "pcx_common.h"

namespace pcx {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int hip_status(hipError_t e, const char* what) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return PCX_EHIP;
}

}  // namespace pcx

extern "C" int pcx_version(void) { return 100; }

extern "C" int pcx_last_error(char* buf, size_t n) {
    size_t len = strlen(pcx::g_err);
    if (buf && n) {
        size_t c = len < n - 1 ? len : n - 1;
        memcpy(buf, pcx::g_err, c);
        buf[c] = 0;
    }
    return (int)len;
}
