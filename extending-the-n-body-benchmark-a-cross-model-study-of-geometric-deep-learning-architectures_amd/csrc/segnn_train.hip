// SEGNN training step (trainer.py:233-358: pred = model(graph); loss.backward()) —
// the native operators the training forward and backward are composed of (fp32).
//
// Reference: models/segnn/segnn.py:150-304, models/segnn/o3_building_blocks.py:10-278, e3nn
// BatchNorm / Gate / FullyConnectedTensorProduct.  Every O(3) tensor product of
// SEGNN (l <= 1) is written in one canonical form:
//   S_in  = [XS | sum_k XV[k] * Y3[:, k]]                     (rows x (Ks + Kv))
//   Zs    = S_in Ws^T,  Zv[k] = XV[k] Wv^T                      (MFMA GEMMs)
//   scalar outputs  OS = Zs[:, :Ms] + b                  (gated: c_silu SiLU(.))
//   vector outputs  OV[k] = Y3[:, k] * Zs[:, NSc + w] + Zv[k]  (gated: * c_sig sigmoid(Zs[:, Ms + w] + b))
// with the e3nn path constants and the SH prefactors folded into Ws / Wv on the host (segnn.py
// train_matrices), so the training forward is: GEMM (nbx_gemm_f32), the TP pre / post elementwise
// kernels, e3nn batch-statistic BatchNorm, and row gathers / segment sums for message passing; the
// backward is the same operators transposed.  Reductions (bias / BatchNorm / weight gradients,
// aggregation) run in a fixed order: the training step is bit-reproducible.
#include <algorithm>
#include <cstring>

#include "nbx_internal.h"
#include "tp_fused.h"   // bf16x3 split helpers (tp_split3, SplitP, mfma32x32)

namespace {

using nbx::kC_SIGMOID;
using nbx::kC_SILU;

typedef float floatx16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------- GEMM (fp32 MFMA)
// C[m][n] (+)= sum_k A(m, k) B(k, n);  A(m, k) = TA ? A[k lda + m] : A[m lda + k],
// B(k, n) = TB ? B[n ldb + k] : B[k ldb + n].  Block tile 64 x 64, K step 32, four waves of a 32 x 32
// v_mfma_f32_32x32x2_f32 tile each; the next K tile is loaded into registers (float4 along the
// contiguous dimension when VEC: 16-byte aligned operands and leading dimensions) while the current
// one is multiplied from LDS.  The training GEMMs are small (a B=64 batch: 320-3840 rows), so the
// grid is split along K until it holds ~256 blocks of >= 4 K steps (gemm_splits): each z writes its
// partial tile into `part` [z][M][N] and gemm_reduce_kernel sums them in z order.  (32 x 32 one-wave
// tiles for grids that would not fill the chip measured slower on every training step, r04.)
constexpr int GB = 64, GK = 32;

template <int T>
struct GemmCfg {
    static constexpr int THREADS = (T / 32) * (T / 32) * 64;   // one wave per 32 x 32 quadrant
    static constexpr int H = T * GK / (THREADS * 4);            // float4 groups per thread per operand
};

struct GemmArgs {
    const float* A;
    const float* B;
    float* C;
    float* part;
    int64_t M, N, K, lda, ldb, ldc;
    int64_t kchunk;   // K range per split
    float beta;
    int ones;         // NBX_GEMM_B_ONES: op(B)'s last column (n = N - 1) is ones, not memory
    int tail;         // NBX_GEMM_ONES_TAIL: C's last column is stored as a row after the M x (N - 1) block
    // two-level rows (nbx_gemm_f32_grouped): row r of a row-major operand with outer stride o != 0 sits
    // at (r / rdiv) o + (r % rdiv) ld -- the (2l + 1) rows of degree l of every node of an
    // [nodes][(lmax + 1)^2][C] array as one [nodes (2l + 1)][C] operand (SO3_LinearV2)
    int64_t rdiv, oa, ob, oc;
    const float* bias;   // nbx_gemm_f32_grouped: C(r, n) += bias[n] (NULL: none)
};

__device__ __forceinline__ int64_t row_off(int64_t r, int64_t ld, int64_t outer, int64_t rdiv) {
    return outer ? (r / rdiv) * outer + (r % rdiv) * ld : r * ld;
}

// address of C(r, c): row-major with leading dimension ldc (two-level rows when oc != 0), except that
// under NBX_GEMM_ONES_TAIL the last column (c = N - 1) is the contiguous vector C + M ldc (a weight
// gradient and its bias gradient then both leave the GEMM contiguous)
__device__ __forceinline__ float* c_at(float* C, int64_t ldc, int64_t oc, int64_t rdiv, int64_t M, int64_t N, int tail,
                                       int64_t r, int64_t c) {
    return (tail && c == N - 1) ? C + M * ldc + r : C + row_off(r, ldc, oc, rdiv) + c;
}

// one 64 x 64 output tile (bx, by) of K split bz of nz (the body of gemm_f32_kernel and of the
// grouped gemm_f32_batched_kernel)
template <bool TA, bool TB, bool VEC, int T = GB>
__device__ __forceinline__ void gemm_tile(const GemmArgs& g, int bx, int by, int bz, int nz, float (&As)[2][GK][T + 4],
                                          float (&Bs)[2][GK][T + 4]) {
    constexpr int THREADS = GemmCfg<T>::THREADS, H = GemmCfg<T>::H, Q4 = T / 4;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int64_t m0 = (int64_t)by * T, n0 = (int64_t)bx * T;
    const int64_t k_lo = (int64_t)bz * g.kchunk;
    const int64_t k_hi = std::min<int64_t>(g.K, k_lo + g.kchunk);
    const int wm = (wave & 1) * 32, wn = (wave >> 1) * 32;
    float ra[H][4], rb[H][4];
    // four consecutive elements along the contiguous dimension: (row, col) of the first, its stride
    auto load4 = [&](const float* base, int64_t ld, int64_t outer, int64_t r, int64_t c, int64_t rmax, int64_t cmax,
                     float (&v)[4]) {
        // elements base[row(r) + c + j], valid while r < rmax and c + j < cmax
        const int64_t ro = row_off(r, ld, outer, g.rdiv);
        if (r < rmax && c + 3 < cmax && VEC) {
            const float4 q = *reinterpret_cast<const float4*>(base + ro + c);
            v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (r < rmax && c + j < cmax) ? base[ro + c + j] : 0.f;
        }
    };
    // float4 group q = t + THREADS h of a K step: [M][K] / [N][K] operands row q / 8, k 4 (q % 8);
    // [K][M] / [K][N] operands k q / Q4, column 4 (q % Q4)
    auto load = [&](int64_t k0) {
#pragma unroll
        for (int h = 0; h < H; ++h) {
            const int q = t + THREADS * h;
            if (TA) load4(g.A, g.lda, g.oa, k0 + q / Q4, m0 + (q % Q4) * 4, k_hi, g.M, ra[h]);   // [K][M]
            else load4(g.A, g.lda, g.oa, m0 + (q >> 3), k0 + (q & 7) * 4, g.M, k_hi, ra[h]);    // [M][K]
            const int64_t bn = TB ? n0 + (q >> 3) : n0 + (q % Q4) * 4, bk = TB ? k0 + (q & 7) * 4 : k0 + q / Q4;
            if (TB) load4(g.B, g.ldb, g.ob, bn, bk, g.N - g.ones, k_hi, rb[h]);   // [N][K]
            else load4(g.B, g.ldb, g.ob, bk, bn, k_hi, g.N - g.ones, rb[h]);      // [K][N]
            if (g.ones && n0 + T >= g.N) {   // the appended column of ones (block-uniform test)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const bool one = TB ? (bn == g.N - 1 && bk + j < k_hi) : (bn + j == g.N - 1 && bk < k_hi);
                    if (one) rb[h][j] = 1.f;
                }
            }
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int h = 0; h < H; ++h) {
            const int q = t + THREADS * h;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (TA) As[buf][q / Q4][(q % Q4) * 4 + j] = ra[h][j];
                else As[buf][(q & 7) * 4 + j][q >> 3] = ra[h][j];
                if (TB) Bs[buf][(q & 7) * 4 + j][q >> 3] = rb[h][j];
                else Bs[buf][q / Q4][(q % Q4) * 4 + j] = rb[h][j];
            }
        }
    };
    floatx16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    const int64_t nk = (k_hi - k_lo + GK - 1) / GK;
    if (nk > 0) {
        load(k_lo);
        store(0);
        __syncthreads();
        for (int64_t it = 0; it < nk; ++it) {
            const int buf = (int)(it & 1);
            if (it + 1 < nk) load(k_lo + (it + 1) * GK);
#pragma unroll
            for (int kk = 0; kk < GK; kk += 2) {
                const float a = As[buf][kk + (lane >> 5)][wm + (lane & 31)];
                const float b = Bs[buf][kk + (lane >> 5)][wn + (lane & 31)];
                acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
            }
            if (it + 1 < nk) store(buf ^ 1);
            __syncthreads();
        }
    }
    // 32x32 accumulator: register i -> row 8 (i / 4) + 4 (lane / 32) + i % 4, column lane % 32
    const int64_t col = n0 + wn + (lane & 31);
    if (col >= g.N) return;
    const bool split = nz > 1;
    float* out = split ? g.part + (int64_t)bz * g.M * g.N : g.C;
    const int64_t ld = split ? g.N : g.ldc;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int64_t row = m0 + wm + 8 * (i >> 2) + 4 * (lane >> 5) + (i & 3);
        if (row >= g.M) continue;
        float* p = split ? out + row * ld + col : c_at(out, ld, g.oc, g.rdiv, g.M, g.N, g.tail, row, col);
        const float v = (!split && g.bias) ? acc[i] + g.bias[col] : acc[i];
        *p = (!split && g.beta != 0.f) ? v + g.beta * *p : v;
    }
}

template <bool TA, bool TB, bool VEC, int T = GB>
__global__ __launch_bounds__(GemmCfg<T>::THREADS) void gemm_f32_kernel(GemmArgs g) {
    __shared__ float As[2][GK][T + 4];
    __shared__ float Bs[2][GK][T + 4];
    gemm_tile<TA, TB, VEC, T>(g, (int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z, (int)gridDim.z, As, Bs);
}

// Up to GMAXP independent GEMMs in one launch (a tensor product's scalar-row and vector-plane GEMMs,
// its four backward GEMMs): block b belongs to the problem whose block range holds it; the operand
// orders (TA, TB) and the float4 path are per problem (block-uniform branches).
constexpr int GMAXP = 8;
struct GemmBatch {
    GemmArgs g[GMAXP];
    int mode[GMAXP];      // bit 0 TA, bit 1 TB, bit 2 VEC
    int tx[GMAXP], ty[GMAXP], nz[GMAXP];
    int first[GMAXP + 1];
    int count;
};

template <int T>
__global__ __launch_bounds__(GemmCfg<T>::THREADS) void gemm_f32_batched_kernel(GemmBatch b) {
    __shared__ float As[2][GK][T + 4];
    __shared__ float Bs[2][GK][T + 4];
    const int blk = (int)blockIdx.x;
    int p = 0;
#pragma unroll
    for (int i = 1; i < GMAXP; ++i)
        if (i < b.count && blk >= b.first[i]) p = i;
    const int local = blk - b.first[p], txy = b.tx[p] * b.ty[p];
    const int bz = local / txy, r = local - bz * txy, by = r / b.tx[p], bx = r - by * b.tx[p];
    const GemmArgs& g = b.g[p];
    switch (b.mode[p]) {
        case 0: gemm_tile<false, false, false, T>(g, bx, by, bz, b.nz[p], As, Bs); break;
        case 1: gemm_tile<true, false, false, T>(g, bx, by, bz, b.nz[p], As, Bs); break;
        case 2: gemm_tile<false, true, false, T>(g, bx, by, bz, b.nz[p], As, Bs); break;
        case 3: gemm_tile<true, true, false, T>(g, bx, by, bz, b.nz[p], As, Bs); break;
        case 4: gemm_tile<false, false, true, T>(g, bx, by, bz, b.nz[p], As, Bs); break;
        case 5: gemm_tile<true, false, true, T>(g, bx, by, bz, b.nz[p], As, Bs); break;
        case 6: gemm_tile<false, true, true, T>(g, bx, by, bz, b.nz[p], As, Bs); break;
        default: gemm_tile<true, true, true, T>(g, bx, by, bz, b.nz[p], As, Bs); break;
    }
}

// the split-K sums of every split problem of a batch in one launch (z order, as gemm_reduce_kernel)
struct ReduceBatch {
    const float* part[GMAXP];
    float* C[GMAXP];
    int64_t M[GMAXP], N[GMAXP], ldc[GMAXP];
    int64_t rdiv[GMAXP], oc[GMAXP];
    const float* bias[GMAXP];
    int splits[GMAXP], tail[GMAXP];
    float beta[GMAXP];
    int64_t first[GMAXP + 1];   // first element of each problem in the flattened index
    int count;
};

// sum_z part[z * MN + e] for z = 0 .. splits - 1, added in z order (bit-identical to the plain loop)
// with the loads issued 8 at a time: a serial load -> add chain paid one full memory latency per split
__device__ __forceinline__ float splitk_sum(const float* __restrict__ part, int splits, int64_t MN, int64_t e) {
    float s = 0.f;
    int z = 0;
    for (; z + 8 <= splits; z += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(z + u) * MN + e];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
    }
    float v[7];
    const int rem = splits - z;
#pragma unroll
    for (int u = 0; u < 7; ++u) v[u] = u < rem ? part[(int64_t)(z + u) * MN + e] : 0.f;
#pragma unroll
    for (int u = 0; u < 7; ++u)
        if (u < rem) s += v[u];
    return s;
}

__global__ void gemm_reduce_batched_kernel(ReduceBatch b) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= b.first[b.count]) return;
    int p = 0;
#pragma unroll
    for (int q = 1; q < GMAXP; ++q)
        if (q < b.count && i >= b.first[q]) p = q;
    const int64_t e = i - b.first[p], N = b.N[p], MN = b.M[p] * N;
    const int64_t r = e / N, c = e - r * N;
    const float s0 = splitk_sum(b.part[p], b.splits[p], MN, e);
    const float s = b.bias[p] ? s0 + b.bias[p][c] : s0;
    float* q = c_at(b.C[p], b.ldc[p], b.oc[p], b.rdiv[p], b.M[p], N, b.tail[p], r, c);
    *q = b.beta[p] != 0.f ? s + b.beta[p] * *q : s;
}

__global__ void gemm_reduce_kernel(const float* __restrict__ part, int splits, int64_t M, int64_t N,
                                   float* __restrict__ C, int64_t ldc, float beta, int tail) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= M * N) return;
    const int64_t r = i / N, c = i - r * N;
    const float s = splitk_sum(part, splits, M * N, i);
    float* p = c_at(C, ldc, 0, 1, M, N, tail, r, c);
    *p = beta != 0.f ? s + beta * *p : s;
}

// ---------------------------------------------------------------- GEMM on the bf16x3 split MFMA
// The large C = A B^T products (NBX_GEMM_TRANS_B on plain rows, one K split: EquiformerV2 lmax 6's
// SO(2) convolutions, 24 320 edge rows, K 448..1536).  Each fp32 operand fragment is split into three
// bf16 parts as it leaves the LDS (tp_fused.h tp_split3: x = hi + mid + lo within 2^-27 |x|) and a
// product is the fp32 sum of the six leading cross terms on v_mfma_f32_32x32x16_bf16 (SplitP<1>,
// smallest first): fp32-level accuracy at up to 2.7x the fp32 MFMA rate (12 x 32 cycles per
// 32 x 32 x 32 step against 16 x 64).  Tile 128 x 128, K step 32, four waves of 64 x 64 (2 x 2 MFMA
// tiles, 24 MFMAs per 16-deep step against 8 fragment splits); both operands are K-contiguous, so the
// LDS holds fp32 rows [row][X3P] (144-byte pitch: a lane's 8 consecutive k are two conflict-free
// ds_read_b128), one buffer, 36 KB.  The 128-wide tile halves the operand re-reads of a 64-wide one,
// which bound it (profiles/r06/gemm_x3/: SO(2) conv 1 group 1 328 us fp32, 1 092 us at 64 x 64, 868 us
// here; splitting once while staging into [part][row] bf16 rows needed 60 KB and ran 1 781 us).
// NBX_GEMM_X3=0 keeps every problem on the fp32 kernel (A/B).
constexpr int X3P = GK + 4;
constexpr int X3T = 128;   // block tile X3T x X3T, four waves of 64 x 64 (2 x 2 MFMA tiles each)

__device__ __forceinline__ void gemm_x3_tile(const GemmArgs& g, int bx, int by, float (&As)[X3T][X3P],
                                             float (&Bs)[X3T][X3P]) {
    using SP = nbx::SplitP<1>;
    constexpr int S = X3T / 64, L = X3T / 32;   // MFMA tiles per wave and dimension; float4s per operand
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int64_t m0 = (int64_t)by * X3T, n0 = (int64_t)bx * X3T;
    const int wm = (wave & 1) * (X3T / 2), wn = (wave >> 1) * (X3T / 2);
    const int r = t >> 3, k4 = (t & 7) * 4;   // this thread stages rows r + 32 h, k4 .. k4 + 3
    float4 a[L], b[L];
    auto ld4 = [&](const float* base, int64_t ld, int64_t row, int64_t rmax, int64_t k, float4& v) {
        if (row < rmax && k + 3 < g.K) {
            v = *reinterpret_cast<const float4*>(base + row * ld + k);
        } else {
            float e[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) e[j] = (row < rmax && k + j < g.K) ? base[row * ld + k + j] : 0.f;
            v = make_float4(e[0], e[1], e[2], e[3]);
        }
    };
    auto load = [&](int64_t k0) {
#pragma unroll
        for (int h = 0; h < L; ++h) {
            ld4(g.A, g.lda, m0 + r + 32 * h, g.M, k0 + k4, a[h]);
            ld4(g.B, g.ldb, n0 + r + 32 * h, g.N, k0 + k4, b[h]);
        }
    };
    floatx16 acc[S][S];
#pragma unroll
    for (int i = 0; i < S; ++i)
#pragma unroll
        for (int j = 0; j < S; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    const int64_t nk = (g.K + GK - 1) / GK;
    if (nk > 0) load(0);
    // one LDS buffer: stage K step it, barrier, request step it + 1, multiply, barrier.  (Two steps in
    // flight: 236 VGPRs under launch bounds (256, 2) and 1.33x slower; profiles/r06/gemm_x3/.)
    for (int64_t it = 0; it < nk; ++it) {
#pragma unroll
        for (int h = 0; h < L; ++h) {
            *reinterpret_cast<float4*>(&As[r + 32 * h][k4]) = a[h];
            *reinterpret_cast<float4*>(&Bs[r + 32 * h][k4]) = b[h];
        }
        __syncthreads();
        if (it + 1 < nk) load((it + 1) * GK);
#pragma unroll
        for (int kk = 0; kk < GK; kk += 16) {
            const int kr = kk + 8 * (lane >> 5);
            nbx::bf16x8 fa[S][3], fb[S][3];
#pragma unroll
            for (int i = 0; i < S; ++i) {
                const float* pa = &As[wm + 32 * i + (lane & 31)][kr];
                const float* pb = &Bs[wn + 32 * i + (lane & 31)][kr];
                nbx::tp_split3(*reinterpret_cast<const float4*>(pa), *reinterpret_cast<const float4*>(pa + 4),
                               fa[i][0], fa[i][1], fa[i][2]);
                nbx::tp_split3(*reinterpret_cast<const float4*>(pb), *reinterpret_cast<const float4*>(pb + 4),
                               fb[i][0], fb[i][1], fb[i][2]);
            }
#pragma unroll
            for (int u = 0; u < SP::NT; ++u)
#pragma unroll
                for (int i = 0; i < S; ++i)
#pragma unroll
                    for (int j = 0; j < S; ++j) acc[i][j] = nbx::mfma32x32(fa[i][SP::TA[u]], fb[j][SP::TB[u]], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < S; ++j) {
        const int64_t col = n0 + wn + 32 * j + (lane & 31);
        if (col >= g.N) continue;
        const float bias = g.bias ? g.bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < S; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int64_t row = m0 + wm + 32 * i + 8 * (e >> 2) + 4 * (lane >> 5) + (e & 3);
                if (row >= g.M) continue;
                float* p = g.C + row * g.ldc + col;
                const float v = g.bias ? acc[i][j][e] + bias : acc[i][j][e];
                *p = g.beta != 0.f ? v + g.beta * *p : v;
            }
    }
}

// the problems of a GemmBatch that are all bf16x3-eligible (gemm_x3_ok; tx / ty count X3T tiles); the
// row blocks of each problem are dealt to the XCDs in groups (block l runs on XCD l % 8 under
// round-robin dispatch): XCD x owns row blocks x, x + 8, ... and walks each one's column tiles, so its
// L2 fetches those A rows once
__global__ __launch_bounds__(256) void gemm_x3_batched_kernel(GemmBatch b) {
    __shared__ float As[X3T][X3P];
    __shared__ float Bs[X3T][X3P];
    const int blk = (int)blockIdx.x;
    int p = 0;
#pragma unroll
    for (int i = 1; i < GMAXP; ++i)
        if (i < b.count && blk >= b.first[i]) p = i;
    const int l = blk - b.first[p], tx = b.tx[p], ty = b.ty[p];
    const int full = (ty / 8) * 8 * tx;   // blocks of the complete 8-row-block groups
    int by, bx;
    if (l < full) {
        const int x = l % 8, j = l / 8;
        by = (j / tx) * 8 + x;
        bx = j % tx;
    } else {
        by = (ty / 8) * 8 + (l - full) / tx;
        bx = (l - full) % tx;
    }
    gemm_x3_tile(b.g[p], bx, by, As, Bs);
}

int64_t gemm_tiles(int64_t M, int64_t N, int T) { return ((M + T - 1) / T) * ((N + T - 1) / T); }

// bf16x3 kernel eligibility: C = A B^T on plain rows, float4-aligned operands, one K split, and large
// enough for the MFMA rate to matter (K >= 64, >= 2^30 multiply-adds; no training-step GEMM qualifies;
// the radial layer 24 320 x 2 304 x 64 143 -> 126 us),
// and at least 96 columns (a 64-column problem would leave half of each 128-wide tile idle: the radial
// output layer 24 320 x 64 x 1152 ran 69 -> 91 us)
bool gemm_x3_ok(int32_t flags, const GemmArgs& g, int splits, bool vec) {
    static const bool on = !(getenv("NBX_GEMM_X3") && getenv("NBX_GEMM_X3")[0] == '0');
    return on && flags == NBX_GEMM_TRANS_B && splits == 1 && vec && g.rdiv == 1 && !g.oa && !g.ob && !g.oc &&
           !g.ones && !g.tail && g.K >= 64 && g.N >= 96 && (double)g.M * g.N * g.K >= 1073741824.0;
}

int gemm_splits(int64_t M, int64_t N, int64_t K, int T) {
    const int64_t tiles = gemm_tiles(M, N, T);
    if (tiles >= 256) return 1;
    const int64_t by_grid = (256 + tiles - 1) / tiles, by_k = K / (4 * GK);
    return (int)std::max<int64_t>(1, std::min<int64_t>(std::min(by_grid, by_k), 64));
}

// ---------------------------------------------------------------- TP pre / post
__global__ void tp_prep_kernel(int64_t rows, int Ks, int Kv, const float* __restrict__ XS, int64_t ldxs,
                               const float* __restrict__ XV, int64_t pvs, const float* __restrict__ Y3,
                               float* __restrict__ S) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int W = Ks + Kv;
    if (i >= rows * W) return;
    const int64_t r = i / W;
    const int c = (int)(i - r * W);
    float v;
    if (c < Ks) {
        v = XS[r * ldxs + c];
    } else {
        const int j = c - Ks;
        const float* y = Y3 + 3 * r;
        v = XV[r * Kv + j] * y[0] + XV[pvs + r * Kv + j] * y[1] + XV[2 * pvs + r * Kv + j] * y[2];
    }
    S[i] = v;
}

// dXS = dS[:, :Ks] (written); dXV[k] += Y3[:, k] * dS[:, Ks:] (accumulated onto the GEMM part)
__global__ void tp_prep_bwd_kernel(int64_t rows, int Ks, int Kv, const float* __restrict__ dS,
                                   const float* __restrict__ Y3, float* __restrict__ dXS, int64_t lddxs,
                                   float* __restrict__ dXV, int64_t pvs) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int W = Ks + Kv;
    if (i >= rows * W) return;
    const int64_t r = i / W;
    const int c = (int)(i - r * W);
    const float d = dS[i];
    if (c < Ks) {
        if (dXS) dXS[r * lddxs + c] = d;
    } else {
        const int j = c - Ks;
        const float* y = Y3 + 3 * r;
#pragma unroll
        for (int k = 0; k < 3; ++k) dXV[k * pvs + r * Kv + j] += y[k] * d;
    }
}

struct TpPost {
    int64_t rows;
    int Ms, Nt, gate;     // NSc = Ms + (gate ? Nt : 0) scalar columns of Zs, then Nt t columns
    const float* Zs;      // [rows][NSc + Nt]
    const float* Zv;      // [3][rows][Nt]
    const float* Y3;      // [rows][3]
    const float* bias;    // [NSc] or null
    const float* RS;      // residual [rows][Ms] or null
    const float* RV;      // residual [3][rows][Nt] or null
    float* OS;            // [rows][Ms]
    float* OV;            // [3][rows][Nt]
    // backward
    const float* dOS;
    const float* dOV;
    float* dZs;
    float* dZv;
};

__device__ inline float sig_f(float x) { return 1.0f / (1.0f + expf(-x)); }

__global__ void tp_post_kernel(TpPost p) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int W = p.Ms + p.Nt;
    if (i >= p.rows * W) return;
    const int64_t r = i / W;
    const int c = (int)(i - r * W);
    const int nsc = p.Ms + (p.gate ? p.Nt : 0), ldz = nsc + p.Nt;
    if (c < p.Ms) {
        float x = p.Zs[r * ldz + c] + (p.bias ? p.bias[c] : 0.f);
        if (p.gate) x = kC_SILU * x * sig_f(x);
        if (p.RS) x += p.RS[r * p.Ms + c];
        p.OS[r * p.Ms + c] = x;
        return;
    }
    const int w = c - p.Ms;
    const int64_t pv = p.rows * p.Nt;
    const float t = p.Zs[r * ldz + nsc + w];
    const float* y = p.Y3 + 3 * r;
    const float g = p.gate ? kC_SIGMOID * sig_f(p.Zs[r * ldz + p.Ms + w] + p.bias[p.Ms + w]) : 1.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int64_t o = k * pv + r * p.Nt + w;
        float v = g * (y[k] * t + p.Zv[o]);
        if (p.RV) v += p.RV[o];
        p.OV[o] = v;
    }
}

__global__ void tp_post_bwd_kernel(TpPost p) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int W = p.Ms + p.Nt;
    if (i >= p.rows * W) return;
    const int64_t r = i / W;
    const int c = (int)(i - r * W);
    const int nsc = p.Ms + (p.gate ? p.Nt : 0), ldz = nsc + p.Nt;
    if (c < p.Ms) {
        const float d = p.dOS[r * p.Ms + c];
        float dz = d;
        if (p.gate) {
            const float x = p.Zs[r * ldz + c] + p.bias[c];
            const float s = sig_f(x);
            dz = d * kC_SILU * s * (1.0f + x * (1.0f - s));
        }
        p.dZs[r * ldz + c] = dz;
        return;
    }
    const int w = c - p.Ms;
    const int64_t pv = p.rows * p.Nt;
    const float t = p.Zs[r * ldz + nsc + w];
    const float* y = p.Y3 + 3 * r;
    float g = 1.f, dg = 0.f, sg = 0.f;
    if (p.gate) {
        sg = sig_f(p.Zs[r * ldz + p.Ms + w] + p.bias[p.Ms + w]);
        g = kC_SIGMOID * sg;
    }
    float dt = 0.f;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int64_t o = k * pv + r * p.Nt + w;
        const float dov = p.dOV[o];
        const float dv = g * dov;
        p.dZv[o] = dv;
        dt += y[k] * dv;
        if (p.gate) dg += dov * (y[k] * t + p.Zv[o]);
    }
    p.dZs[r * ldz + nsc + w] = dt;
    if (p.gate) p.dZs[r * ldz + p.Ms + w] = dg * kC_SIGMOID * sg * (1.0f - sg);
}

// ---------------------------------------------------------------- column sums (bias gradients)
// out[c] = sum_r X[r][c], fixed order: blocks of CS_ROWS rows -> partial rows -> one pass.  A block
// is 4 waves over 64 columns (lane = column, coalesced row reads); wave w sums rows w, w + 4, ... of
// the block's CS_ROWS in fp64 and the 4 wave sums are added in a fixed order through LDS.  Small row
// blocks keep many blocks in flight at the training batch (320-1280 rows): the first version's
// 256-row serial loop per thread ran 10 blocks and took ~60 us per call.
constexpr int CS_ROWS = 32;   // rows per partial block at the training batch (more rows: cs_rows)
__global__ __launch_bounds__(256) void colsum_partial_kernel(int64_t rows, int cols, const float* __restrict__ X,
                                                             int64_t ld, int rpb, double* __restrict__ part) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.y * 64 + lane;
    const int64_t r0 = (int64_t)blockIdx.x * rpb;
    double s = 0.0;
    if (c < cols) {
        const int64_t r1 = std::min<int64_t>(rows, r0 + rpb);
#pragma unroll 4
        for (int64_t r = r0 + w; r < r1; r += 4) s += (double)X[r * ld + c];
    }
    __shared__ double red[4][64];
    red[w][lane] = s;
    __syncthreads();
    if (w == 0 && c < cols)
        part[(int64_t)blockIdx.x * cols + c] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// rows per partial block: CS_ROWS, or more once that would give over 256 partial rows (large
// operands, e.g. PONITA's edge-orientation rows), so the final pass stays short
int cs_rows(int64_t rows) {
    const int64_t r = std::max<int64_t>(CS_ROWS, (rows + 255) / 256);
    return (int)((r + 3) / 4 * 4);
}

// the partial rows summed in a fixed order: 4 waves x 64 columns, wave w takes partials w, w + 4, ...
__global__ __launch_bounds__(256) void colsum_final_kernel(int nb, int cols, const double* __restrict__ part,
                                                           float* __restrict__ out, int accumulate) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.x * 64 + lane;
    double s = 0.0;
    if (c < cols) {
#pragma unroll 4
        for (int b = w; b < nb; b += 4) s += part[(int64_t)b * cols + c];
    }
    __shared__ double red[4][64];
    red[w][lane] = s;
    __syncthreads();
    if (w == 0 && c < cols) {
        const double t = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
        out[c] = accumulate ? out[c] + (float)t : (float)t;
    }
}

// ---------------------------------------------------------------- e3nn BatchNorm, batch statistics
// S [rows][M] (0e channels), V [3][rows][M] (1o channels).  Forward partial sums per block of BN_ROWS
// rows: (sum s, sum s^2, sum |v|^2); backward: (sum dy_s, sum dy_s * xhat, sum dy_v . v).  Same shape
// as colsum_partial_kernel: 4 waves x 64 channels, fixed-order combination.
constexpr int BN_ROWS = 32;
__global__ __launch_bounds__(256) void bn_partial_kernel(int64_t rows, int M, const float* __restrict__ S,
                                                         const float* __restrict__ V, const float* __restrict__ dS,
                                                         const float* __restrict__ dV, const float* __restrict__ save,
                                                         double* __restrict__ part) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int c = blockIdx.y * 64 + lane;
    const int64_t r0 = (int64_t)blockIdx.x * BN_ROWS;
    const int64_t pv = rows * M;
    double a = 0.0, b = 0.0, e = 0.0;
    if (c < M) {
        if (!dS) {
#pragma unroll
            for (int i = w; i < BN_ROWS; i += 4) {
                const int64_t r = r0 + i;
                if (r >= rows) break;
                const double s = S[r * M + c];
                a += s;
                b += s * s;
                const float v0 = V[r * M + c], v1 = V[pv + r * M + c], v2 = V[2 * pv + r * M + c];
                e += (double)v0 * v0 + (double)v1 * v1 + (double)v2 * v2;
            }
        } else {
            const float mu = save[c], inv = save[M + c];
#pragma unroll
            for (int i = w; i < BN_ROWS; i += 4) {
                const int64_t r = r0 + i;
                if (r >= rows) break;
                const double d = dS[r * M + c];
                a += d;
                b += d * (double)((S[r * M + c] - mu) * inv);
#pragma unroll
                for (int k = 0; k < 3; ++k) e += (double)dV[k * pv + r * M + c] * V[k * pv + r * M + c];
            }
        }
    }
    __shared__ double red[3][4][64];
    red[0][w][lane] = a;
    red[1][w][lane] = b;
    red[2][w][lane] = e;
    __syncthreads();
    if (w == 0 && c < M) {
        double* p = part + (int64_t)blockIdx.x * 3 * M;
#pragma unroll
        for (int q = 0; q < 3; ++q) p[q * M + c] = ((red[q][0][lane] + red[q][1][lane]) + red[q][2][lane]) + red[q][3][lane];
    }
}

// save [3][M] = (mu, 1/sqrt(var + eps), 1/sqrt(n + eps)); running stats r <- (1 - m) r + m stat
__global__ void bn_stats_kernel(int nb, int64_t rows_arg, int M, const double* __restrict__ part, float eps,
                                float momentum, float* __restrict__ rmean, float* __restrict__ rvar,
                                float* __restrict__ save, const double* __restrict__ count) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= M) return;
    const double rows = count ? *count : (double)rows_arg;   // SyncBN: the all-reduced row count
    if (!(rows > 0.0)) {
        // no row anywhere (an empty batch without an all-reduced count): no statistics exist; the
        // running statistics stay as they are and the saved coefficients are the identity
        save[c] = 0.f;
        save[M + c] = 1.f;
        save[2 * M + c] = 1.f;
        return;
    }
    double a = 0.0, b = 0.0, e = 0.0;
#pragma unroll 8
    for (int i = 0; i < nb; ++i) {
        const double* p = part + (int64_t)i * 3 * M;
        a += p[c];
        b += p[M + c];
        e += p[2 * M + c];
    }
    const double mu = a / rows;
    double var = b / rows - mu * mu;
    if (var < 0.0) var = 0.0;
    const double n = e / (3.0 * rows);
    save[c] = (float)mu;
    save[M + c] = (float)(1.0 / sqrt(var + (double)eps));
    save[2 * M + c] = (float)(1.0 / sqrt(n + (double)eps));
    if (rmean) {
        rmean[c] = (1.0f - momentum) * rmean[c] + momentum * (float)mu;
        rvar[c] = (1.0f - momentum) * rvar[c] + momentum * (float)var;
        rvar[M + c] = (1.0f - momentum) * rvar[M + c] + momentum * (float)n;
    }
}

__global__ void bn_apply_train_kernel(int64_t rows, int M, const float* __restrict__ S, const float* __restrict__ V,
                                      const float* __restrict__ save, const float* __restrict__ weight,
                                      const float* __restrict__ bias, float* __restrict__ OS, float* __restrict__ OV) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= rows * M) return;
    const int c = (int)(i % M);
    const int64_t pv = rows * M;
    OS[i] = (S[i] - save[c]) * save[M + c] * weight[c] + bias[c];
    const float sv = save[2 * M + c] * weight[M + c];
#pragma unroll
    for (int k = 0; k < 3; ++k) OV[k * pv + i] = V[k * pv + i] * sv;
}

// sums [3][M] of the backward partials -> (dS, dV) and the parameter gradients
__global__ void bn_bwd_apply_kernel(int64_t rows, int M, const float* __restrict__ S, const float* __restrict__ V,
                                    const float* __restrict__ save, const float* __restrict__ weight,
                                    const double* __restrict__ sums, const float* __restrict__ dOS,
                                    const float* __restrict__ dOV, float* __restrict__ dS, float* __restrict__ dV,
                                    const double* __restrict__ count) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= rows * M) return;
    const int c = (int)(i % M);
    const int64_t pv = rows * M;
    const double n = count ? *count : (double)rows;           // SyncBN: means over every rank's rows
    const float mu = save[c], inv = save[M + c], invv = save[2 * M + c];
    const float mdy = (float)(sums[c] / n), mdyx = (float)(sums[M + c] / n);
    const float xh = (S[i] - mu) * inv;
    dS[i] = weight[c] * inv * (dOS[i] - mdy - xh * mdyx);
    const float wv = weight[M + c];
    const float cv = (float)(sums[2 * M + c] / (3.0 * n)) * invv * invv;
#pragma unroll
    for (int k = 0; k < 3; ++k) dV[k * pv + i] = wv * invv * (dOV[k * pv + i] - V[k * pv + i] * cv);
}

// fixed-order sum of the per-block partials into sums [3][M] (+ sums[3M] = rows when count_slot)
__global__ void bn_sum_kernel(int nb, int64_t rows, int M, const double* __restrict__ part, double* __restrict__ sums) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c == 0) sums[3 * M] = (double)rows;
    if (c >= M) return;
    double a = 0.0, b = 0.0, e = 0.0;
#pragma unroll 8
    for (int i = 0; i < nb; ++i) {
        const double* p = part + (int64_t)i * 3 * M;
        a += p[c];
        b += p[M + c];
        e += p[2 * M + c];
    }
    sums[c] = a;
    sums[M + c] = b;
    sums[2 * M + c] = e;
}

__global__ void bn_param_grad_kernel(int nb, int M, const double* __restrict__ part, const float* __restrict__ save,
                                     double* __restrict__ sums, float* __restrict__ dweight,
                                     float* __restrict__ dbias) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= M) return;
    double a = 0.0, b = 0.0, e = 0.0;
#pragma unroll 8
    for (int i = 0; i < nb; ++i) {
        const double* p = part + (int64_t)i * 3 * M;
        a += p[c];
        b += p[M + c];
        e += p[2 * M + c];
    }
    sums[c] = a;
    sums[M + c] = b;
    sums[2 * M + c] = e;
    dbias[c] = (float)a;
    dweight[c] = (float)b;
    dweight[M + c] = (float)(e * save[2 * M + c]);
}

// ---------------------------------------------------------------- gathers and segment sums
// out[r][c] = in[idx[r]][c] per plane (plane = blockIdx.y)
__global__ void gather_rows_kernel(int64_t n, int cols, const int* __restrict__ idx, const float* __restrict__ in,
                                   int64_t ldi, int64_t psi, float* __restrict__ out, int64_t ldo, int64_t pso) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n * cols) return;
    const int64_t r = i / cols, k = blockIdx.y;
    const int c = (int)(i - r * cols);
    out[k * pso + r * ldo + c] = in[k * psi + (int64_t)idx[r] * ldi + c];
}

// out[n][c] (+)= sum_{j in [ptr[n], ptr[n+1])} in[eid[j]][c] per plane, fixed order: one block of 4
// waves per (segment, 64-column slice), lane = column; wave w sums the w-th quarter of the segment
// in CSR order with its row loads issued 8 at a time (long segments -- an embedding-table gradient
// has ~E / #elements rows per segment -- were a serial chain of dependent L2 round trips), then
// the 4 partials are added in wave order through LDS; one grid row (blockIdx.y) per plane
__global__ __launch_bounds__(256) void segment_sum4_kernel(int64_t n, int cols, const int* __restrict__ ptr,
                                                          const int* __restrict__ eid, const float* __restrict__ in,
                                                          int64_t ldi, int64_t psi, float* __restrict__ out,
                                                          int64_t ldo, int64_t pso, int accumulate) {
    __shared__ float part[4][64];
    const int slices = (cols + 63) >> 6;
    const int64_t r = blockIdx.x / slices;
    const int c = (int)(blockIdx.x - r * slices) * 64 + (threadIdx.x & 63), w = threadIdx.x >> 6;
    const int j0 = ptr[r], j1 = ptr[r + 1], len = j1 - j0, q = (len + 3) >> 2;
    const int a = j0 + min(len, w * q), b = j0 + min(len, (w + 1) * q);
    const bool live = c < cols;
    {
        const int64_t k = blockIdx.y;
        const float* src = in + k * psi + (live ? c : 0);
        float s = 0.f;
        int j = a;
        for (; j + 8 <= b; j += 8) {
            int e[8];
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) e[u] = eid[j + u];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = src[(int64_t)e[u] * ldi];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += v[u];
        }
        for (; j < b; ++j) s += src[(int64_t)eid[j] * ldi];
        part[w][threadIdx.x & 63] = s;
        __syncthreads();
        if (w == 0 && live) {
            const int l = threadIdx.x & 63;
            const float t = ((part[0][l] + part[1][l]) + part[2][l]) + part[3][l];
            float* o = out + k * pso + r * ldo + c;
            *o = accumulate ? *o + t : t;
        }
    }
}

// ---------------------------------------------------------------- featurisation (no gradient)
// O3Transform (o3_building_blocks.py:231-278) + catch_isolated_nodes (segnn.py:136-148) on an edge
// list: rel = pos[src] - pos[dst]; node attribute = mean over the incoming edges (dst CSR) of
// SH(rel) + SH(vel), column 0 forced to 1 -> na3 = its l=1 part [V][3];  embedding input
// XS0 = |vel| [V], XV0 [3][V][2] = (pos - mean_xyz(pos), vel) per component; edges:
// rhat [E][3], amf [E][2] = (|rel|, m_src m_dst).
constexpr float kSH1 = nbx::kSH_C1;
__global__ void train_featurize_kernel(int64_t V, int64_t E, const float* __restrict__ pos,
                                       const float* __restrict__ vel, const float* __restrict__ mass,
                                       const int* __restrict__ src, const int* __restrict__ dst,
                                       const int* __restrict__ dptr, const int* __restrict__ deid,
                                       float* __restrict__ na3, float* __restrict__ xs0, float* __restrict__ xv0,
                                       float* __restrict__ rhat, float* __restrict__ amf) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i < E) {
        const int64_t s = src[i], d = dst[i];
        const float rx = pos[3 * s] - pos[3 * d], ry = pos[3 * s + 1] - pos[3 * d + 1];
        const float rz = pos[3 * s + 2] - pos[3 * d + 2];
        const float dist = sqrtf(rx * rx + ry * ry + rz * rz);
        const float inv = 1.0f / fmaxf(dist, 1e-12f);
        rhat[3 * i] = rx * inv;
        rhat[3 * i + 1] = ry * inv;
        rhat[3 * i + 2] = rz * inv;
        amf[2 * i] = dist;
        amf[2 * i + 1] = mass[s] * mass[d];
    }
    if (i < V) {
        const float px = pos[3 * i], py = pos[3 * i + 1], pz = pos[3 * i + 2];
        float ax = 0.f, ay = 0.f, az = 0.f;
        const int j0 = dptr[i], j1 = dptr[i + 1];
        for (int j = j0; j < j1; ++j) {
            const int64_t s = src[deid[j]];
            const float rx = pos[3 * s] - px, ry = pos[3 * s + 1] - py, rz = pos[3 * s + 2] - pz;
            const float inv = 1.0f / fmaxf(sqrtf(rx * rx + ry * ry + rz * rz), 1e-12f);
            ax += kSH1 * rx * inv; ay += kSH1 * ry * inv; az += kSH1 * rz * inv;
        }
        const float cnt = (float)(j1 - j0);
        const float ic = cnt > 0.f ? 1.0f / cnt : 0.f;
        const float vx = vel[3 * i], vy = vel[3 * i + 1], vz = vel[3 * i + 2];
        const float vn = sqrtf(vx * vx + vy * vy + vz * vz);
        const float vd = 1.0f / fmaxf(vn, 1e-12f);
        na3[3 * i] = ax * ic + kSH1 * vx * vd;
        na3[3 * i + 1] = ay * ic + kSH1 * vy * vd;
        na3[3 * i + 2] = az * ic + kSH1 * vz * vd;
        xs0[i] = vn;
        const float mp = (px + py + pz) / 3.0f;   // pos.mean(1): mean over xyz (reference quirk)
        const float pc[3] = {px - mp, py - mp, pz - mp}, vv[3] = {vx, vy, vz};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            xv0[(k * V + i) * 2] = pc[k];
            xv0[(k * V + i) * 2 + 1] = vv[k];
        }
    }
}

unsigned nblk(int64_t n, int t = 256) { return (unsigned)std::max<int64_t>(1, (n + t - 1) / t); }

}  // namespace

// ======================================================================== C ABI (include/nbx.h)
extern "C" int nbx_gemm_f32_workspace_bytes(int64_t M, int64_t N, int64_t K, size_t* bytes) {
    NBX_CHECK_ARG(bytes != nullptr && M >= 0 && N >= 0 && K >= 0, "nbx_gemm_f32_workspace_bytes: bad arguments");
    const int s = gemm_splits(M, N, K, GB);
    *bytes = s > 1 ? (size_t)s * M * N * sizeof(float) : 0;
    return NBX_OK;
}

extern "C" int nbx_gemm_f32(int32_t flags, int64_t M, int64_t N, int64_t K, const float* A, int64_t lda,
                            const float* B, int64_t ldb, float* C, int64_t ldc, float beta, void* workspace,
                            size_t workspace_bytes, void* stream) {
    NBX_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "nbx_gemm_f32: negative size");
    NBX_CHECK_ARG(beta == 0.f || beta == 1.f, "nbx_gemm_f32: beta must be 0 or 1");
    if (M == 0 || N == 0) return NBX_OK;
    NBX_CHECK_ARG(A && B && C, "nbx_gemm_f32: null operand");
    const bool ta = flags & NBX_GEMM_TRANS_A, tb = flags & NBX_GEMM_TRANS_B;
    const int ones = (flags & NBX_GEMM_B_ONES) ? 1 : 0, tail = (flags & NBX_GEMM_ONES_TAIL) ? 1 : 0;
    NBX_CHECK_ARG(!ones || N >= 1, "nbx_gemm_f32: NBX_GEMM_B_ONES needs N >= 1");
    NBX_CHECK_ARG(!tail || ones, "nbx_gemm_f32: NBX_GEMM_ONES_TAIL needs NBX_GEMM_B_ONES");
    NBX_CHECK_ARG(lda >= (ta ? M : K) && ldb >= (tb ? K : N - ones) && ldc >= N - tail,
                  "nbx_gemm_f32: leading dimension too small");
    constexpr int T = GB;
    const int splits = gemm_splits(M, N, K, T);
    const size_t need = splits > 1 ? (size_t)splits * M * N * sizeof(float) : 0;
    NBX_CHECK_ARG(workspace_bytes >= need && (need == 0 || workspace), "nbx_gemm_f32: workspace too small (%zu < %zu)",
                  workspace_bytes, need);
    GemmArgs g{A, B, C, (float*)workspace, M, N, K, lda, ldb, ldc, (K + splits - 1) / splits, beta, ones, tail, 1, 0, 0, 0,
               nullptr};
    g.kchunk = (g.kchunk + GK - 1) / GK * GK;
    const dim3 grid((unsigned)((N + T - 1) / T), (unsigned)((M + T - 1) / T), (unsigned)splits);
    hipStream_t st = (hipStream_t)stream;
    const bool vec = ((uintptr_t)A % 16 == 0) && ((uintptr_t)B % 16 == 0) && lda % 4 == 0 && ldb % 4 == 0;
    if (gemm_x3_ok(flags, g, splits, vec)) {
        GemmBatch gb;
        memset(&gb, 0, sizeof(gb));
        gb.g[0] = g;
        gb.tx[0] = (int)((N + X3T - 1) / X3T);
        gb.ty[0] = (int)((M + X3T - 1) / X3T);
        gb.nz[0] = 1;
        gb.first[1] = gb.tx[0] * gb.ty[0];
        gb.count = 1;
        hipLaunchKernelGGL(gemm_x3_batched_kernel, dim3((unsigned)gb.first[1]), dim3(256), 0, st, gb);
        NBX_LAUNCH_CHECK("gemm_x3");
        return NBX_OK;
    }
    auto launch = [&](auto tile) {
        constexpr int TT = decltype(tile)::value;
        auto go = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(GemmCfg<TT>::THREADS), 0, st, g); };
        if (vec) {
            if (ta && tb) go(gemm_f32_kernel<true, true, true, TT>);
            else if (ta) go(gemm_f32_kernel<true, false, true, TT>);
            else if (tb) go(gemm_f32_kernel<false, true, true, TT>);
            else go(gemm_f32_kernel<false, false, true, TT>);
        } else {
            if (ta && tb) go(gemm_f32_kernel<true, true, false, TT>);
            else if (ta) go(gemm_f32_kernel<true, false, false, TT>);
            else if (tb) go(gemm_f32_kernel<false, true, false, TT>);
            else go(gemm_f32_kernel<false, false, false, TT>);
        }
    };
    launch(std::integral_constant<int, GB>{});
    NBX_LAUNCH_CHECK("gemm_f32");
    if (splits > 1) {
        hipLaunchKernelGGL(gemm_reduce_kernel, dim3(nblk(M * N)), dim3(256), 0, st, (const float*)workspace, splits, M,
                           N, C, ldc, beta, tail);
        NBX_LAUNCH_CHECK("gemm_reduce");
    }
    return NBX_OK;
}

namespace {
// the problems of nbx_gemm_f32_batched (ds = 6 dims each) / nbx_gemm_f32_grouped (ds = 10: + rdiv and
// the outer strides of A, B, C)
struct GroupDims {
    int64_t M, N, K, lda, ldb, ldc, rdiv, oa, ob, oc;
};
GroupDims group_dims(const int64_t* dims, int ds, int i) {
    const int64_t* d = dims + (int64_t)ds * i;
    GroupDims g{d[0], d[1], d[2], d[3], d[4], d[5], 1, 0, 0, 0};
    if (ds == 10) { g.rdiv = d[6]; g.oa = d[7]; g.ob = d[8]; g.oc = d[9]; }
    return g;
}

int gemm_group_ws(const char* name, int32_t count, const int64_t* dims, int ds, size_t* bytes) {
    NBX_CHECK_ARG(bytes != nullptr && dims != nullptr && count >= 1 && count <= GMAXP,
                  "%s_workspace_bytes: bad arguments (count 1..%d)", name, GMAXP);
    size_t n = 0;
    constexpr int T = GB;
    for (int i = 0; i < count; ++i) {
        const GroupDims d = group_dims(dims, ds, i);
        NBX_CHECK_ARG(d.M >= 0 && d.N >= 0 && d.K >= 0, "%s_workspace_bytes: negative size", name);
        const int s = gemm_splits(d.M, d.N, d.K, T);
        if (s > 1) n += ((size_t)s * d.M * d.N + 63) / 64 * 64;
    }
    *bytes = n * sizeof(float);
    return NBX_OK;
}

int gemm_group(const char* name, int32_t count, const int32_t* flags, const int64_t* dims, int ds,
               const float* const* A, const float* const* B, float* const* C, const float* beta,
               const float* const* bias, void* workspace, size_t workspace_bytes, void* stream) {
    NBX_CHECK_ARG(count >= 1 && count <= GMAXP && flags && dims && A && B && C && beta,
                  "%s: bad arguments (count 1..%d)", name, GMAXP);
    GemmBatch gb;
    memset(&gb, 0, sizeof(gb));
    ReduceBatch rb;
    memset(&rb, 0, sizeof(rb));
    int blocks = 0, nred = 0;
    bool x3 = true;   // every problem on the bf16x3 kernel
    size_t ws_off = 0;
    constexpr int T = GB;
    for (int i = 0; i < count; ++i) {
        const GroupDims d = group_dims(dims, ds, i);
        const int64_t M = d.M, N = d.N, K = d.K, lda = d.lda, ldb = d.ldb, ldc = d.ldc;
        const bool ta = flags[i] & NBX_GEMM_TRANS_A, tb = flags[i] & NBX_GEMM_TRANS_B;
        const int ones = (flags[i] & NBX_GEMM_B_ONES) ? 1 : 0, tail = (flags[i] & NBX_GEMM_ONES_TAIL) ? 1 : 0;
        NBX_CHECK_ARG(!tail || ones, "%s: NBX_GEMM_ONES_TAIL needs NBX_GEMM_B_ONES", name);
        NBX_CHECK_ARG(M > 0 && N > 0 && K >= 0, "%s: problem %d: sizes must be positive", name, i);
        NBX_CHECK_ARG(beta[i] == 0.f || beta[i] == 1.f, "%s: beta must be 0 or 1", name);
        NBX_CHECK_ARG(A[i] && B[i] && C[i], "%s: null operand", name);
        NBX_CHECK_ARG(lda >= (ta ? M : K) && ldb >= (tb ? K : N - ones) && ldc >= N - tail,
                      "%s: leading dimension too small", name);
        // two-level rows: rdiv rows of leading dimension ld per outer step, outer >= rdiv ld (no overlap)
        NBX_CHECK_ARG(d.rdiv >= 1 && d.oa >= 0 && d.ob >= 0 && d.oc >= 0, "%s: bad two-level row strides", name);
        NBX_CHECK_ARG((!d.oa || d.oa >= d.rdiv * lda) && (!d.ob || d.ob >= d.rdiv * ldb) &&
                      (!d.oc || d.oc >= d.rdiv * ldc), "%s: outer stride below rdiv x leading dimension", name);
        NBX_CHECK_ARG(!(tail && d.oc), "%s: NBX_GEMM_ONES_TAIL with two-level C rows", name);
        const float* bi = bias ? bias[i] : nullptr;
        NBX_CHECK_ARG(!(bi && ones), "%s: a bias with NBX_GEMM_B_ONES", name);
        const int splits = gemm_splits(M, N, K, T);
        float* part = nullptr;
        if (splits > 1) {
            const size_t need = ((size_t)splits * M * N + 63) / 64 * 64;
            NBX_CHECK_ARG(workspace && (ws_off + need) * sizeof(float) <= workspace_bytes,
                          "%s: workspace too small", name);
            part = (float*)workspace + ws_off;
            ws_off += need;
            rb.part[nred] = part; rb.C[nred] = C[i]; rb.M[nred] = M; rb.N[nred] = N; rb.ldc[nred] = ldc;
            rb.rdiv[nred] = d.rdiv; rb.oc[nred] = d.oc; rb.bias[nred] = bi;
            rb.splits[nred] = splits; rb.tail[nred] = tail; rb.beta[nred] = beta[i];
            rb.first[nred + 1] = rb.first[nred] + M * N;
            ++nred;
        }
        GemmArgs g{A[i], B[i], C[i], part, M, N, K, lda, ldb, ldc, (K + splits - 1) / splits, beta[i], ones, tail,
                   d.rdiv, d.oa, d.ob, d.oc, bi};
        g.kchunk = (g.kchunk + GK - 1) / GK * GK;
        const bool vec = ((uintptr_t)A[i] % 16 == 0) && ((uintptr_t)B[i] % 16 == 0) && lda % 4 == 0 && ldb % 4 == 0 &&
                         d.oa % 4 == 0 && d.ob % 4 == 0;
        gb.g[i] = g;
        x3 = x3 && gemm_x3_ok(flags[i], g, splits, vec);
        gb.mode[i] = (ta ? 1 : 0) | (tb ? 2 : 0) | (vec ? 4 : 0);
        gb.tx[i] = (int)((N + T - 1) / T);
        gb.ty[i] = (int)((M + T - 1) / T);
        gb.nz[i] = splits;
        gb.first[i] = blocks;
        blocks += gb.tx[i] * gb.ty[i] * splits;
        gb.first[i + 1] = blocks;
    }
    gb.count = count;
    rb.count = nred;
    hipStream_t st = (hipStream_t)stream;
    if (x3) {   // (x3 implies no split problem: nred == 0); the grid in X3T x X3T tiles
        int xb = 0;
        for (int i = 0; i < count; ++i) {
            gb.tx[i] = (int)((gb.g[i].N + X3T - 1) / X3T);
            gb.ty[i] = (int)((gb.g[i].M + X3T - 1) / X3T);
            gb.first[i] = xb;
            xb += gb.tx[i] * gb.ty[i];
            gb.first[i + 1] = xb;
        }
        hipLaunchKernelGGL(gemm_x3_batched_kernel, dim3((unsigned)xb), dim3(256), 0, st, gb);
        NBX_LAUNCH_CHECK("gemm_x3_batched");
        return NBX_OK;
    }
    if (count == 1) {   // one problem: the storage-order-specialised kernel (fewer registers than the grouped one)
        const dim3 grid((unsigned)gb.tx[0], (unsigned)gb.ty[0], (unsigned)gb.nz[0]), blk(GemmCfg<GB>::THREADS);
        const GemmArgs& g = gb.g[0];
        switch (gb.mode[0]) {
            case 0: hipLaunchKernelGGL((gemm_f32_kernel<false, false, false, GB>), grid, blk, 0, st, g); break;
            case 1: hipLaunchKernelGGL((gemm_f32_kernel<true, false, false, GB>), grid, blk, 0, st, g); break;
            case 2: hipLaunchKernelGGL((gemm_f32_kernel<false, true, false, GB>), grid, blk, 0, st, g); break;
            case 3: hipLaunchKernelGGL((gemm_f32_kernel<true, true, false, GB>), grid, blk, 0, st, g); break;
            case 4: hipLaunchKernelGGL((gemm_f32_kernel<false, false, true, GB>), grid, blk, 0, st, g); break;
            case 5: hipLaunchKernelGGL((gemm_f32_kernel<true, false, true, GB>), grid, blk, 0, st, g); break;
            case 6: hipLaunchKernelGGL((gemm_f32_kernel<false, true, true, GB>), grid, blk, 0, st, g); break;
            default: hipLaunchKernelGGL((gemm_f32_kernel<true, true, true, GB>), grid, blk, 0, st, g); break;
        }
        NBX_LAUNCH_CHECK("gemm_f32");
    } else {
        hipLaunchKernelGGL(gemm_f32_batched_kernel<GB>, dim3((unsigned)blocks), dim3(GemmCfg<GB>::THREADS), 0, st, gb);
        NBX_LAUNCH_CHECK("gemm_f32_batched");
    }
    if (nred) {
        hipLaunchKernelGGL(gemm_reduce_batched_kernel, dim3(nblk(rb.first[nred])), dim3(256), 0, st, rb);
        NBX_LAUNCH_CHECK("gemm_reduce_batched");
    }
    return NBX_OK;
}
}  // namespace

extern "C" int nbx_gemm_f32_batched_workspace_bytes(int32_t count, const int64_t* dims, size_t* bytes) {
    return gemm_group_ws("nbx_gemm_f32_batched", count, dims, 6, bytes);
}

extern "C" int nbx_gemm_f32_batched(int32_t count, const int32_t* flags, const int64_t* dims, const float* const* A,
                                    const float* const* B, float* const* C, const float* beta, void* workspace,
                                    size_t workspace_bytes, void* stream) {
    return gemm_group("nbx_gemm_f32_batched", count, flags, dims, 6, A, B, C, beta, nullptr, workspace, workspace_bytes,
                      stream);
}

extern "C" int nbx_gemm_f32_grouped_workspace_bytes(int32_t count, const int64_t* dims, size_t* bytes) {
    return gemm_group_ws("nbx_gemm_f32_grouped", count, dims, 10, bytes);
}

extern "C" int nbx_gemm_f32_grouped(int32_t count, const int32_t* flags, const int64_t* dims, const float* const* A,
                                    const float* const* B, float* const* C, const float* beta, const float* const* bias,
                                    void* workspace, size_t workspace_bytes, void* stream) {
    return gemm_group("nbx_gemm_f32_grouped", count, flags, dims, 10, A, B, C, beta, bias, workspace, workspace_bytes,
                      stream);
}

extern "C" int nbx_tp_prep(int64_t rows, int32_t Ks, int32_t Kv, const float* XS, int64_t ldxs, const float* XV,
                           const float* Y3, float* S, void* stream) {
    NBX_CHECK_ARG(rows >= 0 && Ks >= 0 && Kv >= 0 && ldxs >= Ks, "nbx_tp_prep: bad sizes");
    if (rows == 0 || Ks + Kv == 0) return NBX_OK;
    hipLaunchKernelGGL(tp_prep_kernel, dim3(nblk(rows * (Ks + Kv))), dim3(256), 0, (hipStream_t)stream, rows, Ks, Kv,
                       XS, ldxs, XV, rows * Kv, Y3, S);
    NBX_LAUNCH_CHECK("tp_prep");
    return NBX_OK;
}

extern "C" int nbx_tp_prep_backward(int64_t rows, int32_t Ks, int32_t Kv, const float* dS, const float* Y3,
                                    float* dXS, int64_t lddxs, float* dXV, void* stream) {
    NBX_CHECK_ARG(rows >= 0 && Ks >= 0 && Kv >= 0, "nbx_tp_prep_backward: bad sizes");
    if (rows == 0 || Ks + Kv == 0) return NBX_OK;
    NBX_CHECK_ARG(Kv == 0 || dXV, "nbx_tp_prep_backward: null dXV");
    hipLaunchKernelGGL(tp_prep_bwd_kernel, dim3(nblk(rows * (Ks + Kv))), dim3(256), 0, (hipStream_t)stream, rows, Ks,
                       Kv, dS, Y3, dXS, lddxs, dXV, rows * Kv);
    NBX_LAUNCH_CHECK("tp_prep_backward");
    return NBX_OK;
}

extern "C" int nbx_tp_post(int64_t rows, int32_t Ms, int32_t Nt, int32_t gate, const float* Zs, const float* Zv,
                           const float* Y3, const float* bias, const float* RS, const float* RV, float* OS, float* OV,
                           void* stream) {
    NBX_CHECK_ARG(rows >= 0 && Ms >= 0 && Nt >= 0, "nbx_tp_post: bad sizes");
    NBX_CHECK_ARG(!gate || (bias && Ms > 0 && Nt > 0), "nbx_tp_post: a gated TP needs scalars, gates and a bias");
    if (rows == 0 || Ms + Nt == 0) return NBX_OK;
    TpPost p{rows, Ms, Nt, gate, Zs, Zv, Y3, bias, RS, RV, OS, OV, nullptr, nullptr, nullptr, nullptr};
    hipLaunchKernelGGL(tp_post_kernel, dim3(nblk(rows * (Ms + Nt))), dim3(256), 0, (hipStream_t)stream, p);
    NBX_LAUNCH_CHECK("tp_post");
    return NBX_OK;
}

extern "C" int nbx_tp_post_backward(int64_t rows, int32_t Ms, int32_t Nt, int32_t gate, const float* Zs,
                                    const float* Zv, const float* Y3, const float* bias, const float* dOS,
                                    const float* dOV, float* dZs, float* dZv, void* stream) {
    NBX_CHECK_ARG(rows >= 0 && Ms >= 0 && Nt >= 0, "nbx_tp_post_backward: bad sizes");
    NBX_CHECK_ARG(!gate || (bias && Ms > 0 && Nt > 0), "nbx_tp_post_backward: a gated TP needs a bias");
    if (rows == 0 || Ms + Nt == 0) return NBX_OK;
    TpPost p{rows, Ms, Nt, gate, Zs, Zv, Y3, bias, nullptr, nullptr, nullptr, nullptr, dOS, dOV, dZs, dZv};
    hipLaunchKernelGGL(tp_post_bwd_kernel, dim3(nblk(rows * (Ms + Nt))), dim3(256), 0, (hipStream_t)stream, p);
    NBX_LAUNCH_CHECK("tp_post_backward");
    return NBX_OK;
}

extern "C" int nbx_colsum_workspace_bytes(int64_t rows, int32_t cols, size_t* bytes) {
    NBX_CHECK_ARG(bytes && rows >= 0 && cols >= 0, "nbx_colsum_workspace_bytes: bad arguments");
    const int rpb = cs_rows(rows);
    *bytes = (size_t)std::max<int64_t>(1, (rows + rpb - 1) / rpb) * cols * sizeof(double);
    return NBX_OK;
}

extern "C" int nbx_colsum(int64_t rows, int32_t cols, const float* X, int64_t ld, float* out, int32_t accumulate,
                          void* workspace, size_t workspace_bytes, void* stream) {
    NBX_CHECK_ARG(rows >= 0 && cols >= 0 && ld >= cols, "nbx_colsum: bad sizes");
    if (cols == 0) return NBX_OK;
    const int rpb = cs_rows(rows);
    const int nb = (int)std::max<int64_t>(1, (rows + rpb - 1) / rpb);
    NBX_CHECK_ARG(workspace && workspace_bytes >= (size_t)nb * cols * sizeof(double), "nbx_colsum: workspace too small");
    hipStream_t st = (hipStream_t)stream;
    double* part = (double*)workspace;
    if (rows == 0) {
        NBX_HIP(hipMemsetAsync(part, 0, (size_t)cols * sizeof(double), st));
    } else {
        hipLaunchKernelGGL(colsum_partial_kernel, dim3((unsigned)nb, (unsigned)((cols + 63) / 64)), dim3(256), 0, st,
                           rows, cols, X, ld, rpb, part);
        NBX_LAUNCH_CHECK("colsum_partial");
    }
    hipLaunchKernelGGL(colsum_final_kernel, dim3((unsigned)((cols + 63) / 64)), dim3(256), 0, st, nb, cols, part, out,
                       accumulate);
    NBX_LAUNCH_CHECK("colsum_final");
    return NBX_OK;
}

extern "C" int nbx_bn_train_workspace_bytes(int64_t rows, int32_t M, size_t* bytes) {
    NBX_CHECK_ARG(bytes && rows >= 0 && M >= 0, "nbx_bn_train_workspace_bytes: bad arguments");
    *bytes = ((size_t)std::max<int64_t>(1, (rows + BN_ROWS - 1) / BN_ROWS) + 1) * 3 * M * sizeof(double);
    return NBX_OK;
}

extern "C" int nbx_bn_train_forward(int64_t rows, int32_t M, const float* S, const float* V, const float* weight,
                                    const float* bias, float* running_mean, float* running_var, float eps,
                                    float momentum, float* save, float* OS, float* OV, void* workspace,
                                    size_t workspace_bytes, void* stream) {
    NBX_CHECK_ARG(rows > 0 && M > 0, "nbx_bn_train_forward: need rows > 0 and M > 0");
    const int nb = (int)((rows + BN_ROWS - 1) / BN_ROWS);
    NBX_CHECK_ARG(workspace && workspace_bytes >= (size_t)(nb + 1) * 3 * M * sizeof(double),
                  "nbx_bn_train_forward: workspace too small");
    hipStream_t st = (hipStream_t)stream;
    double* part = (double*)workspace;
    const unsigned cb = (unsigned)((M + 63) / 64);
    hipLaunchKernelGGL(bn_partial_kernel, dim3((unsigned)nb, cb), dim3(256), 0, st, rows, M, S, V, nullptr, nullptr,
                       nullptr, part);
    NBX_LAUNCH_CHECK("bn_partial");
    hipLaunchKernelGGL(bn_stats_kernel, dim3(nblk(M)), dim3(256), 0, st, nb, rows, M, part, eps, momentum, running_mean,
                       running_var, save, (const double*)nullptr);
    NBX_LAUNCH_CHECK("bn_stats");
    hipLaunchKernelGGL(bn_apply_train_kernel, dim3(nblk(rows * M)), dim3(256), 0, st, rows, M, S, V, save, weight, bias,
                       OS, OV);
    NBX_LAUNCH_CHECK("bn_apply_train");
    return NBX_OK;
}

extern "C" int nbx_bn_train_backward(int64_t rows, int32_t M, const float* S, const float* V, const float* weight,
                                     const float* save, const float* dOS, const float* dOV, float* dS, float* dV,
                                     float* dweight, float* dbias, void* workspace, size_t workspace_bytes,
                                     void* stream) {
    NBX_CHECK_ARG(rows > 0 && M > 0, "nbx_bn_train_backward: need rows > 0 and M > 0");
    const int nb = (int)((rows + BN_ROWS - 1) / BN_ROWS);
    NBX_CHECK_ARG(workspace && workspace_bytes >= (size_t)(nb + 1) * 3 * M * sizeof(double),
                  "nbx_bn_train_backward: workspace too small");
    hipStream_t st = (hipStream_t)stream;
    double* part = (double*)workspace;
    double* sums = part + (size_t)nb * 3 * M;
    const unsigned cb = (unsigned)((M + 63) / 64);
    hipLaunchKernelGGL(bn_partial_kernel, dim3((unsigned)nb, cb), dim3(256), 0, st, rows, M, S, V, dOS, dOV, save, part);
    NBX_LAUNCH_CHECK("bn_partial(bwd)");
    hipLaunchKernelGGL(bn_param_grad_kernel, dim3(nblk(M)), dim3(256), 0, st, nb, M, part, save, sums, dweight, dbias);
    NBX_LAUNCH_CHECK("bn_param_grad");
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(nblk(rows * M)), dim3(256), 0, st, rows, M, S, V, save, weight, sums,
                       dOS, dOV, dS, dV, (const double*)nullptr);
    NBX_LAUNCH_CHECK("bn_bwd_apply");
    return NBX_OK;
}

// ---- SyncBN training (sharded train-mode BatchNorm): the caller all-reduces the sums between the calls
extern "C" int nbx_bn_train_sums(int64_t rows, int32_t M, const float* S, const float* V, const float* dOS,
                                 const float* dOV, const float* save, double* sums, void* workspace,
                                 size_t workspace_bytes, void* stream) {
    // rows == 0 (an empty shard of a sharded batch): zero sums and a zero count, so every rank still
    // reaches the caller's all-reduce
    NBX_CHECK_ARG(rows >= 0 && M > 0 && sums, "nbx_bn_train_sums: need rows >= 0, M > 0 and sums");
    NBX_CHECK_ARG(!dOS == !dOV && (!dOS || save), "nbx_bn_train_sums: the backward sums need dOS, dOV and save");
    const int nb = (int)((rows + BN_ROWS - 1) / BN_ROWS);
    NBX_CHECK_ARG(rows == 0 || (workspace && workspace_bytes >= (size_t)(nb + 1) * 3 * M * sizeof(double)),
                  "nbx_bn_train_sums: workspace too small");
    hipStream_t st = (hipStream_t)stream;
    double* part = (double*)workspace;
    if (rows > 0) {
        hipLaunchKernelGGL(bn_partial_kernel, dim3((unsigned)nb, (unsigned)((M + 63) / 64)), dim3(256), 0, st, rows, M,
                           S, V, dOS, dOV, save, part);
        NBX_LAUNCH_CHECK("bn_partial(sums)");
    }
    hipLaunchKernelGGL(bn_sum_kernel, dim3(nblk(M)), dim3(256), 0, st, nb, rows, M, part, sums);
    NBX_LAUNCH_CHECK("bn_sum");
    return NBX_OK;
}

extern "C" int nbx_bn_train_apply(int64_t rows, int32_t M, const float* S, const float* V, const float* weight,
                                  const float* bias, const double* sums, float* running_mean, float* running_var,
                                  float eps, float momentum, float* save, float* OS, float* OV, void* stream) {
    // rows == 0: the statistics (and the running-stat update) from the all-reduced sums, no rows to apply
    NBX_CHECK_ARG(rows >= 0 && M > 0 && sums, "nbx_bn_train_apply: need rows >= 0, M > 0 and sums");
    hipStream_t st = (hipStream_t)stream;
    hipLaunchKernelGGL(bn_stats_kernel, dim3(nblk(M)), dim3(256), 0, st, 1, rows, M, sums, eps, momentum, running_mean,
                       running_var, save, sums + 3 * M);
    NBX_LAUNCH_CHECK("bn_stats(sync)");
    if (rows == 0) return NBX_OK;
    hipLaunchKernelGGL(bn_apply_train_kernel, dim3(nblk(rows * M)), dim3(256), 0, st, rows, M, S, V, save, weight, bias,
                       OS, OV);
    NBX_LAUNCH_CHECK("bn_apply_train(sync)");
    return NBX_OK;
}

extern "C" int nbx_bn_train_param_grads(int32_t M, const float* save, const double* local_sums, double* scratch,
                                        float* dweight, float* dbias, void* stream) {
    NBX_CHECK_ARG(M > 0 && save && local_sums && scratch && dweight && dbias, "nbx_bn_train_param_grads: bad arguments");
    hipLaunchKernelGGL(bn_param_grad_kernel, dim3(nblk(M)), dim3(256), 0, (hipStream_t)stream, 1, M, local_sums, save,
                       scratch, dweight, dbias);
    NBX_LAUNCH_CHECK("bn_param_grad(sync)");
    return NBX_OK;
}

extern "C" int nbx_bn_train_backward_apply(int64_t rows, int32_t M, const float* S, const float* V,
                                           const float* weight, const float* save, const double* sums,
                                           const float* dOS, const float* dOV, float* dS, float* dV, void* stream) {
    NBX_CHECK_ARG(rows >= 0 && M > 0 && sums, "nbx_bn_train_backward_apply: need rows >= 0, M > 0 and sums");
    if (rows == 0) return NBX_OK;
    hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(nblk(rows * M)), dim3(256), 0, (hipStream_t)stream, rows, M, S, V, save,
                       weight, sums, dOS, dOV, dS, dV, sums + 3 * M);
    NBX_LAUNCH_CHECK("bn_bwd_apply(sync)");
    return NBX_OK;
}

extern "C" int nbx_gather_rows(int64_t n, int32_t cols, const int32_t* idx, const float* in, int64_t ld_in,
                               int64_t plane_in, float* out, int64_t ld_out, int64_t plane_out, int32_t planes,
                               void* stream) {
    NBX_CHECK_ARG(n >= 0 && cols >= 0 && planes >= 1 && ld_in >= cols && ld_out >= cols, "nbx_gather_rows: bad sizes");
    if (n == 0 || cols == 0) return NBX_OK;
    hipLaunchKernelGGL(gather_rows_kernel, dim3(nblk(n * cols), (unsigned)planes), dim3(256), 0, (hipStream_t)stream, n,
                       cols, idx, in, ld_in, plane_in, out, ld_out, plane_out);
    NBX_LAUNCH_CHECK("gather_rows");
    return NBX_OK;
}

extern "C" int nbx_segment_sum(int64_t n, int32_t cols, const int32_t* ptr, const int32_t* eid, const float* in,
                               int64_t ld_in, int64_t plane_in, float* out, int64_t ld_out, int64_t plane_out,
                               int32_t planes, int32_t accumulate, void* stream) {
    NBX_CHECK_ARG(n >= 0 && cols >= 0 && planes >= 1 && ld_in >= cols && ld_out >= cols, "nbx_segment_sum: bad sizes");
    if (n == 0 || cols == 0) return NBX_OK;
    hipLaunchKernelGGL(segment_sum4_kernel, dim3((unsigned)(n * ((cols + 63) / 64)), (unsigned)planes), dim3(256), 0,
                       (hipStream_t)stream, n, cols, ptr, eid, in, ld_in, plane_in, out, ld_out, plane_out, accumulate);
    NBX_LAUNCH_CHECK("segment_sum");
    return NBX_OK;
}

extern "C" int nbx_segnn_train_featurize(int64_t V, int64_t E, const float* pos, const float* vel, const float* mass,
                                         const int32_t* src, const int32_t* dst, const int32_t* dst_ptr,
                                         const int32_t* dst_eid, float* na3, float* xs0, float* xv0, float* rhat,
                                         float* amf, void* stream) {
    NBX_CHECK_ARG(V >= 1 && E >= 0, "nbx_segnn_train_featurize: bad sizes");
    hipLaunchKernelGGL(train_featurize_kernel, dim3(nblk(std::max(V, E))), dim3(256), 0, (hipStream_t)stream, V, E, pos,
                       vel, mass, src, dst, dst_ptr, dst_eid, na3, xs0, xv0, rhat, amf);
    NBX_LAUNCH_CHECK("segnn_train_featurize");
    return NBX_OK;
}
