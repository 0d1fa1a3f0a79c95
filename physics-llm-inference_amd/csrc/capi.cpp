// C ABI glue of libpli_hip.so: version string and thread-local errors.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

#include "pli_common.h"

namespace pli {

static thread_local char g_err[512] = {0};

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

void clear_error() { g_err[0] = 0; }

int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return int(e);
    }
    return PLI_OK;
}

}  // namespace pli

extern "C" {

const char* pli_version(void) { return "pli_hip 0.1.0 gfx950"; }

const char* pli_last_error(void) { return pli::g_err; }

}  // extern "C"
