// Internal helpers shared by the libnbx translation units (not part of the ABI).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/nbx.h"

namespace nbx {

void set_error(const char* fmt, ...);

// Record `msg` + the HIP error string; returns NBX_E_HIP.
int hip_error(hipError_t e, const char* where);

#define NBX_CHECK_ARG(cond, ...)          \
    do {                                  \
        if (!(cond)) {                    \
            ::nbx::set_error(__VA_ARGS__); \
            return NBX_E_INVAL;           \
        }                                 \
    } while (0)

#define NBX_HIP(expr)                                              \
    do {                                                           \
        hipError_t _e = (expr);                                    \
        if (_e != hipSuccess) return ::nbx::hip_error(_e, #expr);  \
    } while (0)

#define NBX_LAUNCH_CHECK(name) NBX_HIP(hipGetLastError())

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Raise `kernel`'s dynamic-LDS limit to 160 KiB on the current device, once per (kernel, device):
// the attribute is per device, so a process that launches on several devices sets it on each
// (csrc/common.hip).  Returns NBX_OK or NBX_E_HIP.
int lds_limit_160k(const void* kernel);
#define NBX_LDS_160K(kernel)                                                     \
    do {                                                                         \
        if (int _rc = ::nbx::lds_limit_160k((const void*)(kernel))) return _rc;  \
    } while (0)

// Kernel-execution timing for the *_forward_timed entry points: when a start / stop event pair is
// armed, the next NBX_TIMED_LAUNCH records the kernel's own begin / end on them
// (hipExtLaunchKernel: the same interval a profiler's kernel trace reports, without the
// dispatch overhead a hipEventRecord pair around the launch adds); the pair is consumed.
struct ArmedEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};
inline ArmedEvents& armed_events() {
    static thread_local ArmedEvents e;
    return e;
}
// after a launcher that may have returned without launching: record a zero interval instead
inline hipError_t disarm_events(hipStream_t st) {
    ArmedEvents& e = armed_events();
    hipError_t r = hipSuccess;
    if (e.start) {
        r = hipEventRecord(e.start, st);
        if (r == hipSuccess) r = hipEventRecord(e.stop, st);
    }
    e.start = e.stop = nullptr;
    return r;
}
#define NBX_TIMED_LAUNCH(kernel, grid, block, shmem, stream, ...)                                           \
    do {                                                                                                  \
        ::nbx::ArmedEvents& _ae = ::nbx::armed_events();                                                  \
        if (_ae.start) {                                                                                  \
            hipExtLaunchKernelGGL(kernel, grid, block, shmem, stream, _ae.start, _ae.stop, 0, __VA_ARGS__); \
            _ae.start = _ae.stop = nullptr;                                                               \
        } else {                                                                                          \
            hipLaunchKernelGGL(kernel, grid, block, shmem, stream, __VA_ARGS__);                          \
        }                                                                                                 \
    } while (0)

// e3nn / SEGNN constants (oracle/e3nn_lite.py documents their derivation)
constexpr float kSH_C0 = 0.28209479177387814f;   // 1/sqrt(4 pi)
constexpr float kSH_C1 = 0.4886025119029199f;    // sqrt(3/(4 pi))
constexpr float kC_SILU = 1.6791767923989418f;   // normalize2mom(SiLU)
constexpr float kC_SIGMOID = 1.8467055342154763f; // normalize2mom(sigmoid)

// csrc/graph.hip: general graphs as per-destination slot tables (SEGNN, PONITA)
int graph_slots_from_edges(const int64_t* ei, int64_t E, int64_t V, int N, int G, unsigned long long* adj, int* slot,
                           float* deg, int* err, hipStream_t st);
int graph_slots_from_knn(const float* pos, int64_t V, int N, int G, int k, unsigned long long* adj, int* slot,
                         float* deg, int* err, hipStream_t st);

// csrc/comm.hip: sum `count` doubles over the ranks of an RCCL communicator, in place, on `st`
int comm_allreduce_f64(double* buf, int64_t count, void* comm, hipStream_t st);

}  // namespace nbx
