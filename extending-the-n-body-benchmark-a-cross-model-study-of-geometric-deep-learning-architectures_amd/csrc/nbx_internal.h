// Internal helpers shared by the libnbx translation units (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
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

// e3nn / SEGNN constants (oracle/e3nn_lite.py documents their derivation)
constexpr float kSH_C0 = 0.28209479177387814f;   // 1/sqrt(4 pi)
constexpr float kSH_C1 = 0.4886025119029199f;    // sqrt(3/(4 pi))
constexpr float kC_SILU = 1.6791767923989418f;   // normalize2mom(SiLU)
constexpr float kC_SIGMOID = 1.8467055342154763f; // normalize2mom(sigmoid)

}  // namespace nbx
