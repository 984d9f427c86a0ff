// Does v_mfma_f32_16x16x32_f16 keep fp16 subnormal inputs?  A = one subnormal per lane (2^-20) in
// element 0, B = 1.0: the product sum over k must be 2^-20 * (number of subnormal A entries in the row).
// Also checks v_cvt_pk_f16_f32 rounding (RNE vs RTZ) and subnormal outputs of the conversion.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

__global__ void k(float* out, const float* in) {
    const int l = threadIdx.x;
    h8 a, b;
    for (int j = 0; j < 8; ++j) { a[j] = (_Float16)0.0f; b[j] = (_Float16)1.0f; }
    a[0] = (_Float16)in[0];   // subnormal fp16 (2^-20)
    f4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    out[l] = c[0];
    // conversion: 1 + 2^-11 + 2^-13 -> RNE gives 1 + 2^-10, RTZ gives 1
    f2 v = {in[1], in[2]};
    h2 h = __builtin_convertvector(v, h2);
    out[64 + l] = (float)h[0];
    out[128 + l] = (float)h[1];
}

int main() {
    float hin[3] = {0x1p-20f, 1.0f + 0x1p-11f + 0x1p-13f, 0x1p-20f};
    float *din, *dout;
    hipMalloc(&din, sizeof hin);
    hipMalloc(&dout, 192 * sizeof(float));
    hipMemcpy(din, hin, sizeof hin, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dout, din);
    float h[192];
    hipMemcpy(h, dout, sizeof h, hipMemcpyDeviceToHost);
    // row r = 4 (l >> 4) + j ... lane 0 register 0 = row 0, col 0: sum over k of A[0][k] B[k][0]
    // A[row = l & 15][k = 8 (l >> 4) + j]: rows 0..15 each get 4 subnormal entries (one per lane quarter)
    printf("mfma_f16 subnormal input: C[0][0] = %a (kept: %a, flushed: 0x0p+0)\n", h[0], 4 * 0x1p-20f);
    printf("cvt_pk_f16_f32(1 + 2^-11 + 2^-13) = %a (RNE: %a, RTZ: %a)\n", h[64], 1.0f + 0x1p-10f, 1.0f);
    printf("cvt_pk_f16_f32(2^-20) = %a (subnormal kept: %a)\n", h[128], 0x1p-20f);
    return 0;
}
