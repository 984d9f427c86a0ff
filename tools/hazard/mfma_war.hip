// Does a load that returns into the A / B operand registers of a still-pending MFMA change the
// MFMA's result on gfx950?  (The sporadic msg_pre corruption of round 1)
//
// Every lane holds A = B = bf16 1.0 (x8) and runs a chain of v_mfma_f32_16x16x32_bf16 in one
// inline-asm statement (hipcc pads nothing inside it), then a ds_read_b128 / buffer_load_dwordx4
// that overwrites A (or B) with zeros, `GAP` wait states after the last MFMA.  An MFMA that read
// its operands before the load returned adds 32 to every accumulator element; one that read the
// zeros adds 0.  Expected: CHAIN * 32 per element.  The host counts the lanes that differ.
//
//   hipcc --offload-arch=gfx950 -O2 tools/hazard/mfma_war.hip -o /tmp/mfma_war && /tmp/mfma_war
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

#define STR_(x) #x
#define STR(x) STR_(x)
#define MFMA_DEP "v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\t"
#define M32 "v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0\n\t"
#define F32 "v_mfma_f32_32x32x2_f32 %0, %1, %2, %0\n\t"
#define F16 "v_mfma_f32_16x16x4_f32 %0, %1, %2, %0\n\t"
// 64 wait states at the end: every MFMA result is written back before hipcc's code reads %0
#define DRAIN "s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\t"

// The pad (wait states between the last MFMA and the load) is spliced into the asm text by
// the preprocessor: one set of kernels per pad.
#define WAR_KERNELS(NAME, PADSTR)                                                                          \
    template <int KIND>                                                                                    \
    __global__ void NAME(const float* __restrict__ zeros, float* __restrict__ out, float one) {            \
        __shared__ __attribute__((aligned(16))) float lds[256 * 4];                                        \
        const int t = threadIdx.x;                                                                         \
        for (int i = t; i < 256 * 4; i += blockDim.x) lds[i] = 0.f;                                        \
        __syncthreads();                                                                                   \
        bf16x8 a, b;                                                                                       \
        for (int i = 0; i < 8; ++i) { a[i] = (__bf16)one; b[i] = (__bf16)1.0f; } /* distinct registers */    \
        floatx4 acc = {0.f, 0.f, 0.f, 0.f}, acc1 = acc, acc2 = acc, acc3 = acc;                            \
        const unsigned laddr = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)(lds + 4 * t); \
        if constexpr (KIND == 0) {                                                                         \
            asm volatile(MFMA_DEP MFMA_DEP MFMA_DEP MFMA_DEP MFMA_DEP MFMA_DEP MFMA_DEP MFMA_DEP PADSTR     \
                         "ds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)\n\t" DRAIN                           \
                         : "+v"(acc), "+v"(a) : "v"(b), "v"(laddr) : "memory");                            \
        } else if constexpr (KIND == 1) {                                                                  \
            asm volatile(MFMA_DEP MFMA_DEP MFMA_DEP MFMA_DEP MFMA_DEP MFMA_DEP MFMA_DEP MFMA_DEP PADSTR     \
                         "ds_read_b128 %2, %3\n\ts_waitcnt lgkmcnt(0)\n\t" DRAIN                           \
                         : "+v"(acc), "+v"(b), "+v"(a) : "v"(laddr) : "memory");                           \
        } else if constexpr (KIND == 2) {                                                                  \
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %4, %5, %0\n\t"                                     \
                         "v_mfma_f32_16x16x32_bf16 %1, %4, %5, %1\n\t"                                     \
                         "v_mfma_f32_16x16x32_bf16 %2, %4, %5, %2\n\t"                                     \
                         "v_mfma_f32_16x16x32_bf16 %3, %4, %5, %3\n\t"                                     \
                         "v_mfma_f32_16x16x32_bf16 %0, %4, %5, %0\n\t"                                     \
                         "v_mfma_f32_16x16x32_bf16 %1, %4, %5, %1\n\t"                                     \
                         "v_mfma_f32_16x16x32_bf16 %2, %4, %5, %2\n\t"                                     \
                         "v_mfma_f32_16x16x32_bf16 %3, %4, %5, %3\n\t" PADSTR                              \
                         "ds_read_b128 %4, %6\n\ts_waitcnt lgkmcnt(0)\n\t" DRAIN                           \
                         : "+v"(acc), "+v"(acc1), "+v"(acc2), "+v"(acc3), "+v"(a) : "v"(b), "v"(laddr)     \
                         : "memory");                                                                      \
        } else if constexpr (KIND == 3) {                                                                  \
            const __amdgpu_buffer_rsrc_t rs =                                                              \
                __builtin_amdgcn_make_buffer_rsrc((void*)zeros, (short)0, 0x7FFFFFF0, 0x00020000);         \
            const unsigned goff = 16u * (blockIdx.x * blockDim.x + t);                                     \
            asm volatile(MFMA_DEP MFMA_DEP MFMA_DEP MFMA_DEP MFMA_DEP MFMA_DEP MFMA_DEP MFMA_DEP PADSTR     \
                         "buffer_load_dwordx4 %1, %3, %4, 0 offen\n\ts_waitcnt vmcnt(0)\n\t" DRAIN         \
                         : "+v"(acc), "+v"(a) : "v"(b), "v"(goff), "s"(rs) : "memory");                    \
        } else if constexpr (KIND == 4) {                                                                  \
            asm volatile(MFMA_DEP PADSTR "ds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)\n\t" DRAIN          \
                         : "+v"(acc), "+v"(a) : "v"(b), "v"(laddr) : "memory");                            \
        } else if constexpr (KIND == 5) {                                                                  \
            floatx16 c16 = {};                                                                             \
            asm volatile(M32 M32 M32 M32 M32 M32 M32 M32 PADSTR                                            \
                         "ds_read_b128 %2, %3\n\ts_waitcnt lgkmcnt(0)\n\t" DRAIN                           \
                         : "+v"(c16), "+v"(a), "+v"(b) : "v"(laddr) : "memory");                           \
            acc = floatx4{c16[0], c16[1], c16[2], c16[3]};                                                 \
        } else if constexpr (KIND == 6) {                                                                  \
            floatx16 c16 = {};                                                                             \
            float fa = one, fb = 1.0f;                                                                     \
            asm volatile(F32 F32 F32 F32 F32 F32 F32 F32 PADSTR                                            \
                         "ds_read_b32 %2, %3\n\ts_waitcnt lgkmcnt(0)\n\t" DRAIN                            \
                         : "+v"(c16), "+v"(fa), "+v"(fb) : "v"(laddr) : "memory");                         \
            acc = floatx4{c16[0], c16[1], c16[2], c16[3]};                                                 \
        } else if constexpr (KIND == 7) {                                                                  \
            float fa = one, fb = 1.0f;                                                                     \
            asm volatile(F16 F16 F16 F16 F16 F16 F16 F16 PADSTR                                            \
                         "ds_read_b32 %2, %3\n\ts_waitcnt lgkmcnt(0)\n\t" DRAIN                            \
                         : "+v"(acc), "+v"(fa), "+v"(fb) : "v"(laddr) : "memory");                         \
        } else if constexpr (KIND == 8) {                                                                  \
            floatx16 c16 = {};                                                                             \
            asm volatile(M32 M32 M32 M32 M32 M32 M32 M32 PADSTR                                            \
                         "ds_read_b128 %1, %3\n\ts_waitcnt lgkmcnt(0)\n\t" DRAIN                           \
                         : "+v"(c16), "+v"(a), "+v"(b) : "v"(laddr) : "memory");                           \
            acc = floatx4{c16[0], c16[1], c16[2], c16[3]};                                                 \
        } else if constexpr (KIND == 9) {                                                                  \
            floatx16 c16 = {};                                                                             \
            float fa = one, fb = 1.0f;                                                                     \
            asm volatile(F32 F32 F32 F32 F32 F32 F32 F32 PADSTR                                            \
                         "ds_read_b32 %1, %3\n\ts_waitcnt lgkmcnt(0)\n\t" DRAIN                            \
                         : "+v"(c16), "+v"(fa), "+v"(fb) : "v"(laddr) : "memory");                         \
            acc = floatx4{c16[0], c16[1], c16[2], c16[3]};                                                 \
        } else {                                                                                           \
            float fa = one, fb = 1.0f;                                                                     \
            asm volatile(F16 F16 F16 F16 F16 F16 F16 F16 PADSTR                                            \
                         "ds_read_b32 %1, %3\n\ts_waitcnt lgkmcnt(0)\n\t" DRAIN                            \
                         : "+v"(acc), "+v"(fa), "+v"(fb) : "v"(laddr) : "memory");                         \
        }                                                                                                  \
        floatx4 r = acc + acc1 + acc2 + acc3;                                                              \
        float* o = out + 4 * ((size_t)blockIdx.x * blockDim.x + t);                                        \
        o[0] = r[0]; o[1] = r[1]; o[2] = r[2]; o[3] = r[3];                                                \
    }

WAR_KERNELS(war_gap0, "")
WAR_KERNELS(war_gap1, "s_nop 0\n\t")
WAR_KERNELS(war_gap2, "s_nop 1\n\t")
WAR_KERNELS(war_gap3, "s_nop 2\n\t")
WAR_KERNELS(war_gap4, "s_nop 3\n\t")
WAR_KERNELS(war_gap8, "s_nop 7\n\t")
WAR_KERNELS(war_gap16, "s_nop 15\n\t")
WAR_KERNELS(war_gap32, "s_nop 15\n\ts_nop 15\n\t")
WAR_KERNELS(war_gap64, "s_nop 15\n\ts_nop 15\n\ts_nop 15\n\ts_nop 15\n\t")

typedef void (*war_fn)(const float*, float*, float);

long run(war_fn k, const char* what, int gap, float expect, const float* zeros, float* dout, int blocks) {
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, zeros, dout, 1.0f);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return -1; }
    std::vector<float> h((size_t)blocks * 256 * 4);
    (void)hipMemcpy(h.data(), dout, h.size() * 4, hipMemcpyDeviceToHost);
    long bad = 0, lanes = (long)blocks * 256;
    float lo = 1e30f, hi = -1e30f;
    for (long l = 0; l < lanes; ++l) {
        bool ok = true;
        for (int e = 0; e < 4; ++e) {
            const float v = h[4 * l + e];
            ok &= v == expect;
            lo = v < lo ? v : lo;
            hi = v > hi ? v : hi;
        }
        bad += !ok;
    }
    printf("%-60s gap %2d states: %8ld / %ld lanes wrong (values %g .. %g, expected %g)\n", what, gap, bad, lanes,
           lo, hi, expect);
    return bad;
}

int main(int argc, char** argv) {
    const int blocks = 4096;
    float *zeros, *dout;
    (void)hipMalloc(&zeros, (size_t)blocks * 256 * 16);
    (void)hipMemset(zeros, 0, (size_t)blocks * 256 * 16);
    (void)hipMalloc(&dout, (size_t)blocks * 256 * 16);
    const char* names[11] = {"16x16x32 bf16 dependent chain x8, ds_read_b128 -> A",
                             "16x16x32 bf16 dependent chain x8, ds_read_b128 -> B",
                             "16x16x32 bf16 4 independent accs x2, ds_read_b128 -> A",
                             "16x16x32 bf16 dependent chain x8, buffer_load_dwordx4 -> A",
                             "16x16x32 bf16 single MFMA, ds_read_b128 -> A",
                             "32x32x16 bf16 dependent chain x8, ds_read_b128 -> B",
                             "32x32x2 f32 dependent chain x8, ds_read_b32 -> B",
                             "16x16x4 f32 dependent chain x8, ds_read_b32 -> B",
                             "32x32x16 bf16 dependent chain x8, ds_read_b128 -> A",
                             "32x32x2 f32 dependent chain x8, ds_read_b32 -> A",
                             "16x16x4 f32 dependent chain x8, ds_read_b32 -> A"};
    const float expect[11] = {256.f, 256.f, 256.f, 256.f, 32.f, 128.f, 16.f, 32.f, 128.f, 16.f, 32.f};
#define ROW(K) {K<0>, K<1>, K<2>, K<3>, K<4>, K<5>, K<6>, K<7>, K<8>, K<9>, K<10>}
    war_fn k[9][11] = {ROW(war_gap0), ROW(war_gap1), ROW(war_gap2), ROW(war_gap3), ROW(war_gap4),
                       ROW(war_gap8), ROW(war_gap16), ROW(war_gap32), ROW(war_gap64)};
    const int gaps[9] = {0, 1, 2, 3, 4, 8, 16, 32, 64};
    const int maxg = argc > 1 ? atoi(argv[1]) : 9;   // number of gap values to run
    for (int rep = 0; rep < 2; ++rep)
        for (int v = 0; v < 11; ++v)
            for (int g = 0; g < maxg; ++g) run(k[g][v], names[v], gaps[g], expect[v], zeros, dout, blocks);
    (void)hipFree(zeros);
    (void)hipFree(dout);
    return 0;
}
