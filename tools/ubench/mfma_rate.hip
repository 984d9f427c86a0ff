// Micro-benchmark: issue rate of v_mfma_f32_16x16x4_f32 / 32x32x2 with A/B in registers,
// NCH independent accumulator chains, WPS waves per SIMD.  Prints cycles per MFMA per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

template <int NCH>
__global__ void k16(float* out, int iters, unsigned long long* cyc) {
    floatx4 acc[NCH];
    for (int j = 0; j < NCH; ++j) acc[j] = floatx4{0, 0, 0, 0};
    float a = threadIdx.x * 1e-3f, b = 1e-3f;
    __syncthreads();
    unsigned long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int j = 0; j < NCH; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
    }
    unsigned long long t1 = clock64();
    float r = 0;
    for (int j = 0; j < NCH; ++j) r += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NCH>
__global__ void k32(float* out, int iters, unsigned long long* cyc) {
    floatx16 acc[NCH];
    for (int j = 0; j < NCH; ++j) for (int e = 0; e < 16; ++e) acc[j][e] = 0;
    float a = threadIdx.x * 1e-3f, b = 1e-3f;
    __syncthreads();
    unsigned long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int j = 0; j < NCH; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j], 0, 0, 0);
    }
    unsigned long long t1 = clock64();
    float r = 0;
    for (int j = 0; j < NCH; ++j) r += acc[j][0];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class F>
void run(const char* name, F kern, int threads, int nmfma_per_iter) {
    float* out;
    unsigned long long* cyc;
    const int blocks = 256, iters = 200;
    hipMalloc(&out, sizeof(float) * blocks * threads);
    hipMalloc(&cyc, sizeof(unsigned long long) * blocks);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, iters, cyc);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, out, iters, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long h[256];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double avg = 0; for (int i = 0; i < blocks; ++i) avg += h[i]; avg /= blocks;
    printf("%-28s threads %4d: %.1f cycles per MFMA per wave, kernel %.3f ms\n", name, threads,
           avg / (iters * (double)nmfma_per_iter), ms);
    hipFree(out); hipFree(cyc);
}

int main() {
    for (int threads : {256, 512}) {   // 1 or 2 waves per SIMD (one block per CU)
        run("16x16x4 f32, 1 chain", k16<1>, threads, 8);
        run("16x16x4 f32, 2 chains", k16<2>, threads, 16);
        run("16x16x4 f32, 6 chains", k16<6>, threads, 48);
        run("32x32x2 f32, 1 chain", k32<1>, threads, 8);
        run("32x32x2 f32, 3 chains", k32<3>, threads, 24);
    }
    return 0;
}
