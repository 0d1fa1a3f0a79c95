// C ABI glue of libpli_hip.so: version string and thread-local errors.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "pli_common.h"

namespace pli {

static thread_local char g_err[512] = {0};
// kernels launched by the calling thread's current entry-point call, in order
// ('+'-separated; reset with the error message when a call starts)
static thread_local char g_route[512] = {0};

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

void clear_error() {
    g_err[0] = 0;
    g_route[0] = 0;
}

// debug mode (PLI_SYNC=1 or HIP_LAUNCH_BLOCKING=1 in the environment, or
// pli_debug_sync(1)): every
// launch is followed by hipDeviceSynchronize + hipGetLastError, so a kernel
// that faults or fails is reported by the entry point that launched it, with
// the kernel's name in pli_last_error().  Off by default (the library never
// synchronises); not for use while a stream is being captured into a graph.
static std::atomic<int> g_sync{-1};

static int sync_mode() {
    int m = g_sync.load(std::memory_order_relaxed);
    if (m < 0) {
        // PLI_SYNC=1, or the runtime's own HIP_LAUNCH_BLOCKING=1
        m = 0;
        for (const char* name : {"PLI_SYNC", "HIP_LAUNCH_BLOCKING"}) {
            const char* e = getenv(name);
            if (e && *e && strcmp(e, "0") != 0) m = 1;
        }
        g_sync.store(m, std::memory_order_relaxed);
    }
    return m;
}

int launch_status(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: launch failed: %s", what, hipGetErrorString(e));
        return int(e);
    }
    const size_t n = strlen(g_route);
    snprintf(g_route + n, sizeof(g_route) - n, "%s%s", n ? "+" : "", what);
    if (sync_mode()) {
        e = hipDeviceSynchronize();
        if (e == hipSuccess) e = hipGetLastError();
        if (e != hipSuccess) {
            set_error("%s: kernel failed (PLI_SYNC): %s", what, hipGetErrorString(e));
            return int(e);
        }
    }
    return PLI_OK;
}

// CUs of the stream's device, looked up once per device id (a CPX-partitioned
// or second device of the process gets its own count); 256 if the runtime
// cannot say
int cu_count(hipStream_t stream) {
    static std::atomic<int> cache[64];
    hipDevice_t dev = 0;
    if (hipStreamGetDevice(stream, &dev) != hipSuccess) {
        int d = 0;
        if (hipGetDevice(&d) != hipSuccess) return 256;
        dev = d;
    }
    if (dev < 0 || dev >= 64) return 256;
    int n = cache[dev].load(std::memory_order_relaxed);
    if (n > 0) return n;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev].store(n, std::memory_order_relaxed);
    return n;
}

}  // namespace pli

extern "C" {

const char* pli_version(void) { return "pli_hip 0.1.0 gfx950"; }

const char* pli_last_error(void) { return pli::g_err; }

const char* pli_last_route(void) { return pli::g_route; }

int pli_debug_sync(int mode) {
    const int prev = pli::sync_mode();
    if (mode >= 0) pli::g_sync.store(mode ? 1 : 0, std::memory_order_relaxed);
    return prev;
}

}  // extern "C"
