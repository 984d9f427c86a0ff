// Back-to-back launch cost on one stream (tuning tool): N empty kernels, timed with events,
// plain hipLaunchKernelGGL vs hipExtLaunchKernelGGL(any-order), and after a kernel that writes
// a large buffer (dirty L2) vs not.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>

__global__ void empty_k(int) {}
__global__ void dirty_k(float* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = 1.f;
}
__global__ void small_k(float* p) { if (threadIdx.x < 64) p[blockIdx.x * 64 + threadIdx.x] += 1.f; }

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
int main() {
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float* buf;
    const size_t n = 64ull << 20;   // 256 MB
    CK(hipMalloc(&buf, n * 4));
    const int R = 2000;
    float ms;
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(a, st));
        for (int i = 0; i < R; ++i) hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, st, i);
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        printf("empty 1x64, plain launch:        %.2f us/kernel\n", ms * 1e3 / R);
        CK(hipEventRecord(a, st));
        for (int i = 0; i < R; ++i) hipLaunchKernelGGL(small_k, dim3(48), dim3(256), 0, st, buf);
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        printf("small 48x256 rmw, plain launch:  %.2f us/kernel\n", ms * 1e3 / R);
        CK(hipEventRecord(a, st));
        for (int i = 0; i < R; ++i) hipLaunchKernelGGL(empty_k, dim3(1024), dim3(256), 0, st, i);
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        printf("empty 1024x256, plain launch:    %.2f us/kernel\n", ms * 1e3 / R);
        CK(hipEventRecord(a, st));
        for (int i = 0; i < R; ++i) hipExtLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, st, nullptr, nullptr, hipExtAnyOrderLaunch, i);
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        printf("empty 1x64, any-order launch:    %.2f us/kernel\n", ms * 1e3 / R);
        // dirty L2 then empty: time of (dirty + empty) - dirty alone
        const int D = 50;
        CK(hipEventRecord(a, st));
        for (int i = 0; i < D; ++i) hipLaunchKernelGGL(dirty_k, dim3(2048), dim3(256), 0, st, buf, (size_t)(4u << 20));
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        const float d0 = ms;
        CK(hipEventRecord(a, st));
        for (int i = 0; i < D; ++i) {
            hipLaunchKernelGGL(dirty_k, dim3(2048), dim3(256), 0, st, buf, (size_t)(4u << 20));
            hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, st, i);
        }
        CK(hipEventRecord(b, st));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        printf("dirty(16MB) alone %.2f us; empty after dirty adds %.2f us\n", d0 * 1e3 / D, (ms - d0) * 1e3 / D);
    }
    return 0;
}
