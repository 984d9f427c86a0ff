// Error plumbing and version query for the C ABI.
#include "nbx_internal.h"

namespace nbx {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
}

int hip_error(hipError_t e, const char* where) {
    set_error("%s failed: %s", where, hipGetErrorString(e));
    return NBX_E_HIP;
}

}  // namespace nbx

extern "C" int nbx_abi_version(void) { return NBX_ABI_VERSION; }

extern "C" const char* nbx_last_error(void) { return nbx::g_last_error.c_str(); }
