// Error plumbing and version query for the C ABI.
#include <mutex>
#include <set>
#include <utility>
#include <vector>

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

int lds_limit_160k(const void* kernel) {
    static std::mutex mu;
    static std::set<std::pair<const void*, int>> done;
    // lock-free fast path on every launch after the first: this thread's cache of the (kernel, device)
    // pairs already raised (a few dozen entries, scanned linearly)
    thread_local std::vector<std::pair<const void*, int>> seen;
    int dev = 0;
    NBX_HIP(hipGetDevice(&dev));
    for (const auto& e : seen)
        if (e.first == kernel && e.second == dev) return NBX_OK;
    std::lock_guard<std::mutex> lk(mu);
    if (!done.count({kernel, dev})) {
        NBX_HIP(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        done.insert({kernel, dev});
    }
    seen.emplace_back(kernel, dev);
    return NBX_OK;
}

}  // namespace nbx

extern "C" int nbx_abi_version(void) { return NBX_ABI_VERSION; }

extern "C" const char* nbx_last_error(void) { return nbx::g_last_error.c_str(); }
