// Grouped fp32 GEMM on CDNA4 matrix cores: C[M,N] = A[M,K] * Bt[N,K]^T.
//
// v_mfma_f32_32x32x2_f32 (exact f32, k-ordered fma chain).  Block = 256 threads
// = 4 waves, tile 128 x 96 x 32: wave w owns rows [32w, 32w+32) and all 96
// columns (three 32x32 accumulators).  A and Bt tiles are staged through LDS
// with K contiguous (pitch 36 floats: conflict-free ds_read_b128 for the
// fragment pattern below); the next K-tile is prefetched into registers while
// the current one is consumed.  K is permuted inside a 32-deep tile so that a
// lane reads 16 consecutive k (4 x ds_read_b128): at MFMA step s lane-half h
// supplies k = 16h + s for BOTH operands, which leaves the sum unchanged.
// M, N, K tails are zero-filled; requires K % 4 == 0 and 16-byte aligned rows.
#pragma once
#include "nbx_internal.h"

namespace nbx {

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct GemmProb {
    const float* A;   // [M][lda]
    const float* Bt;  // [N][ldb]
    float* C;         // [M][ldc]
    int M, N, K;
    int lda, ldb, ldc;
    int tiles_n;      // ceil(N / 96)
    int tiles;        // ceil(M / 128) * tiles_n
};

constexpr int kMaxGemmProbs = 4;

struct GemmBatch {
    GemmProb p[kMaxGemmProbs];
    int np;
};

constexpr int GEMM_BM = 128, GEMM_BN = 96, GEMM_BK = 32, GEMM_PITCH = GEMM_BK + 4;

__global__ __launch_bounds__(256) void gemm_f32_kernel(const GemmBatch gb) {
    __shared__ __attribute__((aligned(16))) float As[GEMM_BM * GEMM_PITCH];
    __shared__ __attribute__((aligned(16))) float Bs[GEMM_BN * GEMM_PITCH];

    int bid = blockIdx.x;
    int pi = 0;
    while (pi < gb.np - 1 && bid >= gb.p[pi].tiles) {
        bid -= gb.p[pi].tiles;
        ++pi;
    }
    const GemmProb& P = gb.p[pi];
    const int tm = bid / P.tiles_n, tn = bid - tm * P.tiles_n;
    const int m0 = tm * GEMM_BM, n0 = tn * GEMM_BN;
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63, r = lane & 31, h = lane >> 5;

    float4 ra[4], rb[3];
    auto load_tile = [&](int k0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = t + 256 * i, row = f >> 3, kq = (f & 7) * 4;
            const int m = m0 + row, k = k0 + kq;
            ra[i] = (m < P.M && k < P.K) ? *reinterpret_cast<const float4*>(P.A + (size_t)m * P.lda + k)
                                         : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int f = t + 256 * i, n = f >> 3, kq = (f & 7) * 4;
            const int nn = n0 + n, k = k0 + kq;
            rb[i] = (nn < P.N && k < P.K) ? *reinterpret_cast<const float4*>(P.Bt + (size_t)nn * P.ldb + k)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto store_tile = [&]() {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = t + 256 * i, row = f >> 3, kq = (f & 7) * 4;
            *reinterpret_cast<float4*>(&As[row * GEMM_PITCH + kq]) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int f = t + 256 * i, n = f >> 3, kq = (f & 7) * 4;
            *reinterpret_cast<float4*>(&Bs[n * GEMM_PITCH + kq]) = rb[i];
        }
    };

    floatx16 acc[3];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[j][e] = 0.f;

    const int nk = (P.K + GEMM_BK - 1) / GEMM_BK;
    load_tile(0);
    store_tile();
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) load_tile((kt + 1) * GEMM_BK);
        const float* arow = &As[(32 * wave + r) * GEMM_PITCH + 16 * h];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float4 a4 = *reinterpret_cast<const float4*>(arow + 4 * q);
            float4 b4[3];
#pragma unroll
            for (int j = 0; j < 3; ++j)
                b4[j] = *reinterpret_cast<const float4*>(&Bs[(32 * j + r) * GEMM_PITCH + 16 * h + 4 * q]);
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.x, b4[j].x, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.y, b4[j].y, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.z, b4[j].z, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a4.w, b4[j].w, acc[j], 0, 0, 0);
            }
        }
        __syncthreads();
        if (kt + 1 < nk) {
            store_tile();
            __syncthreads();
        }
    }
    // C/D map of the 32x32 f32 MFMA: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const int col = n0 + 32 * j + r;
        if (col >= P.N) continue;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int row = m0 + 32 * wave + (e & 3) + 8 * (e >> 2) + 4 * h;
            if (row < P.M) P.C[(size_t)row * P.ldc + col] = acc[j][e];
        }
    }
}

inline GemmProb make_prob(const float* A, int lda, const float* Bt, int ldb, float* C, int ldc, int M, int N, int K) {
    GemmProb p;
    p.A = A; p.Bt = Bt; p.C = C;
    p.M = M; p.N = N; p.K = K;
    p.lda = lda; p.ldb = ldb; p.ldc = ldc;
    p.tiles_n = (N + GEMM_BN - 1) / GEMM_BN;
    p.tiles = ((M + GEMM_BM - 1) / GEMM_BM) * p.tiles_n;
    return p;
}

// Launch up to kMaxGemmProbs independent problems in one grid.
inline int gemm_f32(const GemmProb* probs, int np, hipStream_t stream) {
    GemmBatch gb;
    gb.np = 0;
    int total = 0;
    for (int i = 0; i < np; ++i) {
        if (probs[i].M <= 0 || probs[i].N <= 0) continue;
        if (probs[i].K % 4 || probs[i].lda % 4 || probs[i].ldb % 4) {
            set_error("gemm_f32: K, lda, ldb must be multiples of 4");
            return NBX_E_INVAL;
        }
        gb.p[gb.np++] = probs[i];
        total += probs[i].tiles;
    }
    if (gb.np == 0) return NBX_OK;
    hipLaunchKernelGGL(gemm_f32_kernel, dim3(total), dim3(256), 0, stream, gb);
    NBX_HIP(hipGetLastError());
    return NBX_OK;
}

}  // namespace nbx
