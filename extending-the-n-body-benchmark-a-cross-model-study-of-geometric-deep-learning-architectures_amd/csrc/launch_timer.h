// Optional per-launch HIP-event timing of selected kernels, grouped by "kind", on the
// stream the kernels run on (used by the *_forward_timed entry points that bench.py
// reads to compute the live roofline of the dominant kernel).
#pragma once
#include <vector>

#include "nbx_internal.h"

namespace nbx {

struct LaunchTimer {
    static constexpr int KINDS = 8;
    std::vector<hipEvent_t> ev;
    std::vector<int> kind;
    double flops[KINDS] = {};
    double bytes[KINDS] = {};
    int launches[KINDS] = {};

    int begin(hipStream_t st) {
        hipEvent_t a, b;
        NBX_HIP(hipEventCreate(&a));
        NBX_HIP(hipEventCreate(&b));
        ev.push_back(a);
        ev.push_back(b);
        NBX_HIP(hipEventRecord(a, st));
        return NBX_OK;
    }
    int end(hipStream_t st, int k, double fl, double by) {
        NBX_HIP(hipEventRecord(ev.back(), st));
        kind.push_back(k);
        flops[k] += fl;
        bytes[k] += by;
        launches[k] += 1;
        return NBX_OK;
    }
    // waits for the events, sums per kind, releases them
    int collect(float* kind_ms) {
        for (int k = 0; k < KINDS; ++k) kind_ms[k] = 0.f;
        int rc = NBX_OK;
        for (size_t i = 0; i < kind.size(); ++i) {
            float ms = 0.f;
            if (hipEventSynchronize(ev[2 * i + 1]) != hipSuccess ||
                hipEventElapsedTime(&ms, ev[2 * i], ev[2 * i + 1]) != hipSuccess)
                rc = NBX_E_HIP;
            kind_ms[kind[i]] += ms;
        }
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
        ev.clear();
        kind.clear();
        if (rc) set_error("launch timer: event query failed");
        return rc;
    }
};

// run `fn` (returning an NBX status) between a pair of events when a timer is given
template <class F>
int timed(LaunchTimer* tm, hipStream_t st, int k, double fl, double by, F&& fn) {
    if (!tm) return fn();
    if (int rc = tm->begin(st)) return rc;
    if (int rc = fn()) return rc;
    return tm->end(st, k, fl, by);
}

}  // namespace nbx
