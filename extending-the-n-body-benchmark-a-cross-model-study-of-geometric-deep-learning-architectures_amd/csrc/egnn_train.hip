// EGNN-MC training step on the device: a forward that keeps the activations the backward needs, and
// the backward of the whole network (embedding, every _EGNNMessageBlock, both vector heads) to the
// gradient of the persistent kernel's weight blob (include/nbx.h "EGNN-MC persist blob").
//
// Reference: models/egnn_mc/egnn_mc.py:45-295 (the module trained by trainer.py:233-358 through
// loss.backward()), dataloaders/egnn_mc_n_body_dataloader.py:8-56 (node / edge inputs: data, no
// gradient).  The host wraps the pair in a torch.autograd.Function whose input is the blob built
// from the parameters by differentiable ops, so torch routes the blob gradient to every parameter
// and the reference trainer's optimizer / clipping / scheduler run unchanged.
//
// One 512-thread workgroup per system (N <= 8 bodies, E = N (N - 1) edges), fp32 FMA arithmetic
// over LDS-resident activations (the per-system products are 20-56 rows; these are latency-bound
// reductions, not MFMA work).  Saved per system and layer (global scratch):
//   hin [N][H], coord_in [N][4], ZE1 ZEF ZC1 [E][H] (pre-activations), U [E] (coord head before
//   tanh), ZV1 ZN1 AGG [N][H]; after the layers: h [N][H], coord [N][4], per head ZG1 ZG2 [N][H].
// Weight gradients of one workgroup accumulate into its own slice of a partial buffer
// [G][blob] (systems g, g + G, ...); a second kernel sums the G slices (deterministic order).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "nbx_internal.h"

namespace {

constexpr int ET_THREADS = 512;

__device__ inline float et_sig(float z) { return 1.0f / (1.0f + __expf(-z)); }
__device__ inline float et_silu(float z) { return z * et_sig(z); }
__device__ inline float et_dsilu(float z) {
    const float s = et_sig(z);
    return s * (1.0f + z * (1.0f - s));
}

// The block-wide products below give every thread RB = 4 independent rows (accumulation chains)
// of one output column, so each weight load feeds 4 FMAs and the chains overlap their latency.
constexpr int RB = 4;

// Y[r][n] = b[n] + sum_k X[r][k] W[k][n] (W input-major [K][ldw]); Zs (global, optional) gets the
// pre-activation; Y gets act(.) with act 1 = SiLU.  X / Y in LDS.  All threads call.
__device__ __forceinline__ void et_gemm(const float* X, int rows, int ldx, int K, const float* __restrict__ W, int ldw,
                        const float* __restrict__ b, int Nc, float* Y, int ldy, int act, float* Zs) {
    const int rg = (rows + RB - 1) / RB;
    for (int o = threadIdx.x; o < rg * Nc; o += ET_THREADS) {
        const int g = o / Nc, n = o - g * Nc, r0 = g * RB;
        float v[RB];
        const float* x[RB];
#pragma unroll
        for (int j = 0; j < RB; ++j) {
            v[j] = b ? b[n] : 0.f;
            x[j] = X + (r0 + j < rows ? r0 + j : r0) * ldx;
        }
#pragma unroll 16
        for (int k = 0; k < K; ++k) {
            const float w = W[(size_t)k * ldw + n];
#pragma unroll
            for (int j = 0; j < RB; ++j) v[j] = fmaf(x[j][k], w, v[j]);
        }
#pragma unroll
        for (int j = 0; j < RB; ++j) {
            const int r = r0 + j;
            if (r >= rows) break;
            if (Zs) Zs[r * Nc + n] = v[j];
            Y[r * ldy + n] = act == 1 ? et_silu(v[j]) : v[j];
        }
    }
    __syncthreads();
}

// dX[r][k] (+)= sum_n dZ[r][n] W[k][n] (n < Nc; Nc, ldz, ldw multiples of 4, rows 16-byte aligned).
// Thread = one output column k (of RS row ranges when K < 512): W row k is read once, 32 columns at
// a time into registers, and every dZ float4 is an LDS broadcast (all lanes of a wave read the same
// row); 4 rows per pass give 4 independent FMA chains.
constexpr int ET_TC = 4;   // float4 columns of W per register chunk
__device__ __forceinline__ void et_gemm_t(const float* dZ, int rows, int ldz, int Nc, const float* __restrict__ W, int ldw, int K,
                          float* dX, int ldx, bool accumulate) {
    const int RS = K >= ET_THREADS ? 1 : ET_THREADS / K;
    for (int t = threadIdx.x; t < K * RS; t += ET_THREADS) {
        const int k = t % K, part = t / K;
        const int ra = rows * part / RS, rb = rows * (part + 1) / RS;
        const float* w = W + (size_t)k * ldw;
        for (int c0 = 0; c0 < Nc; c0 += 4 * ET_TC) {
            float4 wr[ET_TC];
#pragma unroll
            for (int i = 0; i < ET_TC; ++i)
                wr[i] = c0 + 4 * i < Nc ? *reinterpret_cast<const float4*>(w + c0 + 4 * i) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 1
            for (int r0 = ra; r0 < rb; r0 += 4) {
                float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int i = 0; i < ET_TC; ++i) {
                    if (c0 + 4 * i >= Nc) break;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int r = r0 + j < rb ? r0 + j : rb - 1;
                        const float4 z = *reinterpret_cast<const float4*>(dZ + r * ldz + c0 + 4 * i);
                        v[j] = fmaf(z.x, wr[i].x, fmaf(z.y, wr[i].y, fmaf(z.z, wr[i].z, fmaf(z.w, wr[i].w, v[j]))));
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int r = r0 + j;
                    if (r >= rb) break;
                    float* o = dX + r * ldx + k;
                    *o = (accumulate || c0 > 0) ? *o + v[j] : v[j];
                }
            }
        }
    }
    __syncthreads();
}

// G[k][n] += sum_r X[r][k] dZ[r][n] (k < K), gb[n] += sum_r dZ[r][n]; G / gb global (this workgroup's
// partial slice), X / dZ in LDS or global (K, Nc, ldx, ldz, ldg multiples of 4, rows 16-byte aligned).
// Thread = a 4 x 4 block of G: per row one float4 of X and one of dZ feed 16 FMAs.
__device__ __forceinline__ void et_wgrad(const float* X, int rows, int ldx, int K, const float* dZ, int ldz, int Nc, float* G, int ldg,
                         float* gb, bool first) {
    const int kq = K >> 2, nq = Nc >> 2;
    for (int o = threadIdx.x; o < kq * nq; o += ET_THREADS) {
        const int kb = o / nq, nb = o - kb * nq, k0 = 4 * kb, n0 = 4 * nb;
        float4 a[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int r = 0; r < rows; ++r) {
            const float4 x = *reinterpret_cast<const float4*>(X + r * ldx + k0);
            const float4 z = *reinterpret_cast<const float4*>(dZ + r * ldz + n0);
            const float xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                a[i].x = fmaf(xs[i], z.x, a[i].x);
                a[i].y = fmaf(xs[i], z.y, a[i].y);
                a[i].z = fmaf(xs[i], z.z, a[i].z);
                a[i].w = fmaf(xs[i], z.w, a[i].w);
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float4* g = reinterpret_cast<float4*>(G + (size_t)(k0 + i) * ldg + n0);
            if (first) {   // the workgroup's first system writes its slice (no read-modify-write latency)
                *g = a[i];
            } else {
                float4 c = *g;
                c.x += a[i].x; c.y += a[i].y; c.z += a[i].z; c.w += a[i].w;
                *g = c;
            }
        }
    }
    if (gb)
        for (int n = threadIdx.x; n < Nc; n += ET_THREADS) {
            float v = 0.f;
            for (int r = 0; r < rows; ++r) v += dZ[r * ldz + n];
            gb[n] = first ? v : gb[n] + v;
        }
    __syncthreads();
}

// Sum over the 16 lanes of a DPP row; every lane of the row gets the total (4 VALU adds, no LDS).
__device__ __forceinline__ float et_row_sum16(float v) {
    auto dpp = [](float x, int ctrl) -> float {
        switch (ctrl) {   // (the control must be a compile-time constant)
            case 0: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, true));
            case 1: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, true));
            case 2: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x141, 0xF, 0xF, true));
            default: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x140, 0xF, 0xF, true));
        }
    };
    v += dpp(v, 0);   // quad_perm [1,0,3,2]
    v += dpp(v, 1);   // quad_perm [2,3,0,1]: quad sums
    v += dpp(v, 2);   // row_half_mirror: sums of 8
    v += dpp(v, 3);   // row_mirror: sums of 16
    return v;
}

// One 16-column tile of a register-resident product: Y[r][c0 + c] = sum_q A[r][q] B(q, c0 + c) over the
// contraction q < Q (Q % 4 == 0) for all rows, where lane = (slice sl = lane & 15, column group
// cg = lane >> 4) holds B for its 4 columns and the contraction blocks qb = sl + 16 j in registers
// (loaded once), reads A rows as LDS float4 broadcasts, and the 16 slices of a column group (one DPP
// row) are summed with et_row_sum16; lane sl of the row then owns output (row r0 + sl / 4, column
// 4 cg + sl % 4) of the 4-row pass.  TRANS = false: B(q, n) = W[q][n] (W input-major [Q][ldw]);
// TRANS = true: B(q, n) = W[n][q] (W [ncols][ldw], the transposed product of the backward).
template <int KB, bool TRANS, class Epi>
__device__ __forceinline__ void et_tile(const float* A, int rows, int lda, int Q, const float* __restrict__ W, int ldw,
                                        int c0, int ncols, Epi epi) {
    const int lane = threadIdx.x & 63, sl = lane & 15, cg = lane >> 4;
    const int n0 = c0 + 4 * cg;
    const int qq = Q >> 2;
    float4 w[KB][4];
#pragma unroll
    for (int j = 0; j < KB; ++j) {
        const int qb = sl + 16 * j;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (qb >= qq) { w[j][i] = make_float4(0.f, 0.f, 0.f, 0.f); continue; }
            if constexpr (!TRANS) {
                w[j][i] = *reinterpret_cast<const float4*>(W + (size_t)(4 * qb + i) * ldw + n0);
            } else {   // w[j][i] = (W[n0][4qb + i], W[n0 + 1][4qb + i], ...): 4 column rows, transposed
                const int n = n0 + i < ncols ? n0 + i : ncols - 1;
                w[j][i] = *reinterpret_cast<const float4*>(W + (size_t)n * ldw + 4 * qb);
            }
        }
    }
    for (int r0 = 0; r0 < rows; r0 += 4) {
        float acc[4][4];
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[rr][c] = 0.f;
#pragma unroll
        for (int j = 0; j < KB; ++j) {
            const int qb = sl + 16 * j;
            if (qb >= qq) break;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int r = r0 + rr < rows ? r0 + rr : rows - 1;
                const float4 x = *reinterpret_cast<const float4*>(A + r * lda + 4 * qb);
                if constexpr (!TRANS) {
                    // w[j][i] = W[4qb + i][n0 .. n0 + 3]
                    acc[rr][0] = fmaf(x.x, w[j][0].x, fmaf(x.y, w[j][1].x, fmaf(x.z, w[j][2].x, fmaf(x.w, w[j][3].x, acc[rr][0]))));
                    acc[rr][1] = fmaf(x.x, w[j][0].y, fmaf(x.y, w[j][1].y, fmaf(x.z, w[j][2].y, fmaf(x.w, w[j][3].y, acc[rr][1]))));
                    acc[rr][2] = fmaf(x.x, w[j][0].z, fmaf(x.y, w[j][1].z, fmaf(x.z, w[j][2].z, fmaf(x.w, w[j][3].z, acc[rr][2]))));
                    acc[rr][3] = fmaf(x.x, w[j][0].w, fmaf(x.y, w[j][1].w, fmaf(x.z, w[j][2].w, fmaf(x.w, w[j][3].w, acc[rr][3]))));
                } else {
                    // w[j][c] = W[n0 + c][4qb .. 4qb + 3]
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        acc[rr][c] = fmaf(x.x, w[j][c].x, fmaf(x.y, w[j][c].y, fmaf(x.z, w[j][c].z, fmaf(x.w, w[j][c].w, acc[rr][c]))));
                }
            }
        }
        float mine = 0.f;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const float t = et_row_sum16(acc[rr][c]);
                mine = sl == 4 * rr + c ? t : mine;
            }
        const int r = r0 + (sl >> 2), n = n0 + (sl & 3);
        if (r < rows && n < ncols) epi(r, n, mine);
    }
}

// forward product, H = HT in {32, 64, 128}: Y = act(X W + b) (W input-major [K][HT], K % 4 == 0,
// K <= 2 HT + 8); wave w computes the 16-column tiles w, w + 8, ...
template <int HT>
__device__ __forceinline__ void et_gemm_r(const float* X, int rows, int ldx, int K, const float* __restrict__ W,
                                          const float* __restrict__ b, float* Y, int ldy, int act, float* Zs) {
    constexpr int KB = ((2 * HT + 8) / 4 + 15) / 16;
    for (int t = threadIdx.x >> 6; t < HT / 16; t += ET_THREADS / 64)
        et_tile<KB, false>(X, rows, ldx, K, W, HT, 16 * t, HT, [&](int r, int n, float v) {
            const float z = v + (b ? b[n] : 0.f);
            if (Zs) Zs[r * HT + n] = z;
            Y[r * ldy + n] = act == 1 ? et_silu(z) : z;
        });
    __syncthreads();
}

// backward transposed product, H = HT: dX[r][k] (+)= sum_n dZ[r][n] W[k][n] (n < HT, k < K)
template <int HT>
__device__ __forceinline__ void et_gemm_t_r(const float* dZ, int rows, int ldz, const float* __restrict__ W, int K,
                                            float* dX, int ldx, bool accumulate) {
    constexpr int KB = (HT / 4 + 15) / 16;
    for (int t = threadIdx.x >> 6; t < (K + 15) / 16; t += ET_THREADS / 64)
        et_tile<KB, true>(dZ, rows, ldz, HT, W, HT, 16 * t, K, [&](int r, int k, float v) {
            float* o = dX + r * ldx + k;
            *o = accumulate ? *o + v : v;
        });
    __syncthreads();
}

// forward product: the register-resident form at H = 32 / 64 / 128 (HT), the generic one otherwise
template <int HT>
__device__ __forceinline__ void et_fwd(const float* X, int rows, int ldx, int K, const float* __restrict__ W, int ldw,
                              const float* __restrict__ b, int Nc, float* Y, int ldy, int act, float* Zs) {
    if constexpr (HT > 0) et_gemm_r<HT>(X, rows, ldx, K, W, b, Y, ldy, act, Zs);
    else et_gemm(X, rows, ldx, K, W, ldw, b, Nc, Y, ldy, act, Zs);
}

// transposed product: the register-resident form at H = HT, the generic one otherwise
template <int HT>
__device__ __forceinline__ void et_bwd(const float* dZ, int rows, int ldz, int Nc, const float* __restrict__ W, int ldw,
                                       int K, float* dX, int ldx, bool accumulate) {
    if constexpr (HT > 0) et_gemm_t_r<HT>(dZ, rows, ldz, W, K, dX, ldx, accumulate);
    else et_gemm_t(dZ, rows, ldz, Nc, W, ldw, K, dX, ldx, accumulate);
}

// out[r] = sum_k X[r][k] w[k * ws] for rows r: one wave per row, lanes over k, shuffle sum
__device__ __forceinline__ float et_wave_dot(const float* x, const float* __restrict__ w, int ws, int K) {
    float v = 0.f;
    for (int k = threadIdx.x & 63; k < K; k += 64) v = fmaf(x[k], w[(size_t)k * ws], v);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

struct EgnnTrain {
    const float* blob;      // weights (persist blob layout)
    int L, N, heads, recurrent, norm_diff, use_tanh, H;
    float coords_weight;
    const float* pos; const float* vel; const float* mass;   // [B N 3], [B N 3], [B N]
    int64_t B;
    float* save;            // [B][save_floats]
    int64_t save_floats;
    float* out;             // forward: [B N][3 heads]
    const float* dout;      // backward: dL/dout [B N][3 heads]
    float* gpart;           // backward: [G][blob_floats] partial weight gradients (zeroed by the host)
    int64_t blob_floats;
    unsigned long long* dbg;   // NBX_ET_DEBUG: per-workgroup phase clocks [grid][16] (tuning only)
};

// phase clocks of thread 0 (NBX_ET_DEBUG; every phase ends at a workgroup barrier)
struct EtClock {
    unsigned long long last, acc[16];
    __device__ void start(const EgnnTrain& P) {
        if (P.dbg && threadIdx.x == 0) {
            last = clock64();
            for (int i = 0; i < 16; ++i) acc[i] = 0;
        }
    }
    __device__ void tick(const EgnnTrain& P, int i) {
        if (P.dbg && threadIdx.x == 0) {
            const unsigned long long t = clock64();
            acc[i] += t - last;
            last = t;
        }
    }
    __device__ void flush(const EgnnTrain& P) {
        if (P.dbg && threadIdx.x == 0)
            for (int i = 0; i < 16; ++i) P.dbg[blockIdx.x * 16 + i] = acc[i];
    }
};

// blob offsets (include/nbx.h): embedding [2][H] + b[H]; per layer e0 [2H+8][H] e0b e1 [H][H] e1b
// c0 [H][H] c0b c1w [H] v0 [H][H] v0b v1w [H] v1b [4] n0 [2H][H] n0b n1 [H][H] n1b; per head
// w0 [H+8][H] b0 w1 [H][H] b1 w2 [H][4] b2 [4]
struct LayerOff {
    int64_t e0, e0b, e1, e1b, c0, c0b, c1w, v0, v0b, v1w, v1b, n0, n0b, n1, n1b;
};
__device__ inline LayerOff layer_off(int H, int l) {
    LayerOff o;
    const int64_t LAYER = 8LL * H * H + 16LL * H + 4;
    o.e0 = 3LL * H + l * LAYER;
    o.e0b = o.e0 + (2LL * H + 8) * H;
    o.e1 = o.e0b + H; o.e1b = o.e1 + (int64_t)H * H;
    o.c0 = o.e1b + H; o.c0b = o.c0 + (int64_t)H * H;
    o.c1w = o.c0b + H;
    o.v0 = o.c1w + H; o.v0b = o.v0 + (int64_t)H * H;
    o.v1w = o.v0b + H; o.v1b = o.v1w + H;
    o.n0 = o.v1b + 4; o.n0b = o.n0 + 2LL * H * H;
    o.n1 = o.n0b + H; o.n1b = o.n1 + (int64_t)H * H;
    return o;
}
struct HeadOff {
    int64_t w0, b0, w1, b1, w2, b2;
};
__device__ inline HeadOff head_off(int H, int L, int t) {
    HeadOff o;
    const int64_t LAYER = 8LL * H * H + 16LL * H + 4, HEAD = 2LL * H * H + 14LL * H + 4;
    o.w0 = 3LL * H + L * LAYER + t * HEAD;
    o.b0 = o.w0 + (H + 8LL) * H;
    o.w1 = o.b0 + H; o.b1 = o.w1 + (int64_t)H * H;
    o.w2 = o.b1 + H; o.b2 = o.w2 + 4LL * H;
    return o;
}

// per-system saved layout (floats)
struct SaveOff {
    int64_t layer, hin, cin, ze1, zef, zc1, u, zv1, zn1, agg;   // within a layer
    int64_t hfin, cfin, head, zg1, zg2;                          // after the layers
};
__host__ __device__ inline SaveOff save_off(int N, int H, int L) {
    const int E = N * (N - 1);
    SaveOff s;
    s.hin = 0; s.cin = s.hin + (int64_t)N * H; s.ze1 = s.cin + 4LL * N; s.zef = s.ze1 + (int64_t)E * H;
    s.zc1 = s.zef + (int64_t)E * H; s.u = s.zc1 + (int64_t)E * H; s.zv1 = s.u + ((E + 3) & ~3);
    s.zn1 = s.zv1 + (int64_t)N * H;   // (every block starts 16-byte aligned: float4 access)
    s.agg = s.zn1 + (int64_t)N * H;
    s.layer = s.agg + (int64_t)N * H;
    s.hfin = L * s.layer; s.cfin = s.hfin + (int64_t)N * H;
    s.zg1 = 0; s.zg2 = (int64_t)N * H; s.head = 2LL * N * H;
    return s;
}
__host__ __device__ inline int64_t save_floats(int N, int H, int L, int heads) {
    const SaveOff s = save_off(N, H, L);
    return (s.cfin + 4LL * N + heads * s.head + 3) & ~3LL;
}

// LDS (floats), E = N (N - 1): X [E][2H+8] | dX [E][2H+8] | A B C [E][H] | n0..n4 [N][2H] | small
__host__ __device__ inline size_t train_lds_floats(int N, int H) {
    const int E = N * (N - 1);
    return 2 * (size_t)E * (2 * H + 8) + 3 * (size_t)E * H + 5 * (size_t)N * 2 * H + 64 * 8 + 16 * (size_t)E + 32 * (size_t)N;
}

struct Lds {
    float *X, *dX, *A, *Bq, *Cq, *n0, *n1, *n2, *n3, *n4;
    float *pos0, *coord, *velv, *mass, *ea, *diff, *diffn, *radial, *cd, *vd, *dvd, *dcd, *dcoord, *dpred, *tmp;
};
__device__ inline Lds carve_lds(float* lds, int N, int H) {
    const int E = N * (N - 1);
    Lds s;
    float* p = lds;
    s.X = p; p += (size_t)E * (2 * H + 8);
    s.dX = p; p += (size_t)E * (2 * H + 8);
    s.A = p; p += (size_t)E * H;
    s.Bq = p; p += (size_t)E * H;
    s.Cq = p; p += (size_t)E * H;
    s.n0 = p; p += 2 * N * H;
    s.n1 = p; p += 2 * N * H;
    s.n2 = p; p += 2 * N * H;
    s.n3 = p; p += 2 * N * H;
    s.n4 = p; p += 2 * N * H;
    s.pos0 = p; p += 32;
    s.coord = p; p += 32;
    s.velv = p; p += 32;
    s.mass = p; p += 32;
    s.dcoord = p; p += 32;
    s.dpred = p; p += 64;
    s.vd = p; p += 8;
    s.dvd = p; p += 8;
    s.tmp = p; p += 64;
    s.ea = p; p += 4 * E;
    s.diff = p; p += 3 * E;
    s.diffn = p; p += 3 * E;
    s.radial = p; p += E;
    s.cd = p; p += E;
    s.dcd = p; p += E;
    return s;
}

__device__ inline int e_row(int e, int deg) { return e / deg; }
__device__ inline int e_col(int e, int deg) {
    const int i = e / deg, j = e - i * deg;
    return j < i ? j : j + 1;
}

// node / edge inputs of one system into LDS (egnn_mc_n_body_dataloader.py:8-56)
__device__ void load_system(const EgnnTrain& P, const Lds& s, int64_t sys) {
    const int N = P.N, deg = N - 1, E = N * deg;
    for (int i = threadIdx.x; i < 3 * N; i += ET_THREADS) {
        s.pos0[i] = P.pos[sys * N * 3 + i];
        s.velv[i] = P.vel[sys * N * 3 + i];
    }
    for (int i = threadIdx.x; i < N; i += ET_THREADS) s.mass[i] = P.mass[sys * N + i];
    __syncthreads();
    for (int e = threadIdx.x; e < E; e += ET_THREADS) {
        const int r = e_row(e, deg), c = e_col(e, deg);
        const float dx = s.pos0[3 * r] - s.pos0[3 * c], dy = s.pos0[3 * r + 1] - s.pos0[3 * c + 1],
                    dz = s.pos0[3 * r + 2] - s.pos0[3 * c + 2];
        const float d2 = dx * dx + dy * dy + dz * dz, d = fmaxf(sqrtf(d2), 1e-12f);
        const float hx = dx / d, hy = dy / d, hz = dz / d;
        s.ea[4 * e] = s.mass[r] * s.mass[c];
        s.ea[4 * e + 1] = s.velv[3 * r] * hx + s.velv[3 * r + 1] * hy + s.velv[3 * r + 2] * hz;
        s.ea[4 * e + 2] = s.velv[3 * c] * hx + s.velv[3 * c + 1] * hy + s.velv[3 * c + 2] * hz;
        s.ea[4 * e + 3] = d2;
    }
    __syncthreads();
}

// coord2radial (egnn_mc.py:155-164) of the coordinates in s.coord
__device__ void geometry(const EgnnTrain& P, const Lds& s) {
    const int N = P.N, deg = N - 1, E = N * deg;
    for (int e = threadIdx.x; e < E; e += ET_THREADS) {
        const int r = e_row(e, deg), c = e_col(e, deg);
        float d[3];
        for (int k = 0; k < 3; ++k) d[k] = s.coord[4 * r + k] - s.coord[4 * c + k];
        const float radial = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        const float nrm = P.norm_diff ? fmaxf(sqrtf(radial), 1.0f) : 1.0f;
        for (int k = 0; k < 3; ++k) {
            s.diff[3 * e + k] = d[k];
            s.diffn[3 * e + k] = d[k] / nrm;
        }
        s.radial[e] = radial;
    }
    __syncthreads();
}

// edge input [h_row | h_col | radial, edge_attr, 0 0 0] from h in LDS [N][H]
__device__ void edge_input(const EgnnTrain& P, const Lds& s, const float* h) {
    const int N = P.N, deg = N - 1, E = N * deg, H = P.H, LX = 2 * H + 8;
    for (int o = threadIdx.x; o < E * LX; o += ET_THREADS) {
        const int e = o / LX, k = o - e * LX;
        float v;
        if (k < H) v = h[e_row(e, deg) * H + k];
        else if (k < 2 * H) v = h[e_col(e, deg) * H + k - H];
        else if (k == 2 * H) v = s.radial[e];
        else if (k < 2 * H + 5) v = s.ea[4 * e + k - 2 * H - 1];
        else v = 0.f;
        s.X[o] = v;
    }
    __syncthreads();
}

template <int HT>
__global__ __launch_bounds__(ET_THREADS) void egnn_train_fwd_kernel(const EgnnTrain P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int N = P.N, deg = N - 1, E = N * deg, H = HT > 0 ? HT : P.H, LX = 2 * H + 8;
    const Lds s = carve_lds(lds, N, H);
    const int64_t sys = blockIdx.x;
    const SaveOff so = save_off(N, H, P.L);
    float* sv = P.save + sys * P.save_floats;
    EtClock ck;
    ck.start(P);
    load_system(P, s, sys);
    // embedding: x = [|vel|, mass] (Linear 2 -> H)
    float* h = s.n0;
    for (int o = threadIdx.x; o < N * H; o += ET_THREADS) {
        const int i = o / H, n = o - i * H;
        const float vx = s.velv[3 * i], vy = s.velv[3 * i + 1], vz = s.velv[3 * i + 2];
        h[o] = P.blob[2 * H + n] + sqrtf(vx * vx + vy * vy + vz * vz) * P.blob[n] + s.mass[i] * P.blob[H + n];
    }
    for (int i = threadIdx.x; i < N; i += ET_THREADS)
        for (int k = 0; k < 4; ++k) s.coord[4 * i + k] = k < 3 ? s.pos0[3 * i + k] : 0.f;
    __syncthreads();
    for (int l = 0; l < P.L; ++l) {
        const LayerOff w = layer_off(H, l);
        float* sl = sv + l * so.layer;
        for (int o = threadIdx.x; o < N * H; o += ET_THREADS) sl[so.hin + o] = h[o];
        for (int o = threadIdx.x; o < 4 * N; o += ET_THREADS) sl[so.cin + o] = s.coord[o];
        geometry(P, s);
        edge_input(P, s, h);
        ck.tick(P, 0);
        et_fwd<HT>(s.X, E, LX, LX, P.blob + w.e0, H, P.blob + w.e0b, H, s.A, H, 1, sl + so.ze1);    // E1
        et_fwd<HT>(s.A, E, H, H, P.blob + w.e1, H, P.blob + w.e1b, H, s.Bq, H, 1, sl + so.zef);      // EF
        ck.tick(P, 1);
        et_fwd<HT>(s.Bq, E, H, H, P.blob + w.c0, H, P.blob + w.c0b, H, s.A, H, 1, sl + so.zc1);      // C1
        ck.tick(P, 2);
        for (int e = threadIdx.x >> 6; e < E; e += ET_THREADS / 64) {                              // coord head
            const float u = et_wave_dot(s.A + e * H, P.blob + w.c1w, 1, H);
            if ((threadIdx.x & 63) == 0) {
                sl[so.u + e] = u;
                s.cd[e] = P.use_tanh ? tanhf(u) : u;
            }
        }
        ck.tick(P, 3);
        et_fwd<HT>(h, N, H, H, P.blob + w.v0, H, P.blob + w.v0b, H, s.n1, H, 1, sl + so.zv1);        // V1
        ck.tick(P, 4);
        for (int i = threadIdx.x >> 6; i < N; i += ET_THREADS / 64) {
            const float v = et_wave_dot(s.n1 + i * H, P.blob + w.v1w, 1, H);
            if ((threadIdx.x & 63) == 0) s.vd[i] = P.blob[w.v1b] + v;
        }
        for (int o = threadIdx.x; o < N * H; o += ET_THREADS) {                                   // [h | mean EF]
            const int i = o / H, n = o - i * H;
            float a = 0.f;
            for (int q = 0; q < deg; ++q) a += s.Bq[(i * deg + q) * H + n];
            a = deg > 0 ? a / (float)deg : 0.f;
            sl[so.agg + o] = a;
            s.n2[i * 2 * H + n] = h[o];
            s.n2[i * 2 * H + H + n] = a;
        }
        __syncthreads();
        ck.tick(P, 5);
        et_fwd<HT>(s.n2, N, 2 * H, 2 * H, P.blob + w.n0, H, P.blob + w.n0b, H, s.n3, H, 1, sl + so.zn1);   // N1
        float* hn = h == s.n0 ? s.n4 : s.n0;
        et_fwd<HT>(s.n3, N, H, H, P.blob + w.n1, H, P.blob + w.n1b, H, hn, H, 0, nullptr);
        ck.tick(P, 6);
        for (int o = threadIdx.x; o < 3 * N; o += ET_THREADS) {   // coord_model + velocity term
            const int i = o / 3, k = o - 3 * i;
            float a = 0.f;
            for (int q = 0; q < deg; ++q) {
                const int e = i * deg + q;
                a += fminf(fmaxf(s.diffn[3 * e + k] * s.cd[e], -100.f), 100.f);
            }
            s.tmp[o] = (deg > 0 ? a / (float)deg : 0.f) * P.coords_weight + s.vd[i] * s.velv[o];
        }
        if (P.recurrent)
            for (int o = threadIdx.x; o < N * H; o += ET_THREADS) hn[o] += h[o];
        __syncthreads();
        for (int o = threadIdx.x; o < 3 * N; o += ET_THREADS) s.coord[4 * (o / 3) + o % 3] += s.tmp[o];
        __syncthreads();
        ck.tick(P, 7);
        h = hn;
    }
    for (int o = threadIdx.x; o < N * H; o += ET_THREADS) sv[so.hfin + o] = h[o];
    for (int o = threadIdx.x; o < 4 * N; o += ET_THREADS) sv[so.cfin + o] = s.coord[o];
    // heads: [h | coord - pos, vel, 0 0] -> SiLU -> SiLU -> 3
    const int LH = H + 8;
    for (int o = threadIdx.x; o < N * LH; o += ET_THREADS) {
        const int i = o / LH, k = o - i * LH;
        float v = 0.f;
        if (k < H) v = h[i * H + k];
        else if (k < H + 3) v = s.coord[4 * i + k - H] - s.pos0[3 * i + k - H];
        else if (k < H + 6) v = s.velv[3 * i + k - H - 3];
        s.X[o] = v;
    }
    __syncthreads();
    for (int t = 0; t < P.heads; ++t) {
        const HeadOff w = head_off(H, P.L, t);
        float* sh = sv + so.cfin + 4 * N + t * so.head;
        et_fwd<HT>(s.X, N, LH, LH, P.blob + w.w0, H, P.blob + w.b0, H, s.n1, H, 1, sh + so.zg1);
        et_fwd<HT>(s.n1, N, H, H, P.blob + w.w1, H, P.blob + w.b1, H, s.n2, H, 1, sh + so.zg2);
        for (int o = threadIdx.x >> 6; o < 3 * N; o += ET_THREADS / 64) {
            const int i = o / 3, k = o - 3 * i;
            const float v = et_wave_dot(s.n2 + i * H, P.blob + w.w2 + k, 4, H);
            if ((threadIdx.x & 63) == 0) P.out[(sys * N + i) * 3 * P.heads + 3 * t + k] = P.blob[w.b2 + k] + v;
        }
        __syncthreads();
    }
    ck.tick(P, 8);
    ck.flush(P);
}

template <int HT>
__global__ __launch_bounds__(ET_THREADS) void egnn_train_bwd_kernel(const EgnnTrain P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int N = P.N, deg = N - 1, E = N * deg, H = HT > 0 ? HT : P.H, LX = 2 * H + 8, LH = H + 8;
    const Lds s = carve_lds(lds, N, H);
    const SaveOff so = save_off(N, H, P.L);
    float* G = P.gpart + (int64_t)blockIdx.x * P.blob_floats;
    EtClock ck;
    ck.start(P);
    for (int64_t sys = blockIdx.x; sys < P.B; sys += gridDim.x) {
        const bool first = sys == blockIdx.x;
        const float* sv = P.save + sys * P.save_floats;
        load_system(P, s, sys);
        for (int o = threadIdx.x; o < 3 * N * P.heads; o += ET_THREADS) s.dpred[o] = P.dout[sys * N * 3 * P.heads + o];
        // dh (s.n0) and dcoord start at zero
        float* dh = s.n0;
        for (int o = threadIdx.x; o < N * H; o += ET_THREADS) dh[o] = 0.f;
        for (int o = threadIdx.x; o < 3 * N; o += ET_THREADS) s.dcoord[o] = 0.f;
        // ---- heads
        for (int o = threadIdx.x; o < N * LH; o += ET_THREADS) {   // head input from the saved final state
            const int i = o / LH, k = o - i * LH;
            float v = 0.f;
            if (k < H) v = sv[so.hfin + i * H + k];
            else if (k < H + 3) v = sv[so.cfin + 4 * i + k - H] - s.pos0[3 * i + k - H];
            else if (k < H + 6) v = s.velv[3 * i + k - H - 3];
            s.X[o] = v;
        }
        __syncthreads();
        for (int t = 0; t < P.heads; ++t) {
            const HeadOff w = head_off(H, P.L, t);
            const float* sh = sv + so.cfin + 4 * N + t * so.head;
            // G1 = silu(ZG1) -> n1, G2 = silu(ZG2) -> n2
            for (int o = threadIdx.x; o < N * H; o += ET_THREADS) {
                s.n1[o] = et_silu(sh[so.zg1 + o]);
                s.n2[o] = et_silu(sh[so.zg2 + o]);
            }
            for (int o = threadIdx.x; o < 3 * N; o += ET_THREADS) {   // dpred of this head -> tmp [N][3]
                const int i = o / 3, k = o - 3 * i;
                s.tmp[o] = s.dpred[i * 3 * P.heads + 3 * t + k];
            }
            __syncthreads();
            // pred = G2 W2 + b2: dG2 = dpred W2^T; gW2 += G2^T dpred (3 of 4 columns); gb2
            for (int o = threadIdx.x; o < H * 3; o += ET_THREADS) {
                const int n = o / 3, k = o - 3 * n;
                float v = 0.f;
                for (int i = 0; i < N; ++i) v = fmaf(s.n2[i * H + n], s.tmp[3 * i + k], v);
                G[w.w2 + 4 * n + k] += v;
            }
            for (int k = threadIdx.x; k < 3; k += ET_THREADS) {
                float v = 0.f;
                for (int i = 0; i < N; ++i) v += s.tmp[3 * i + k];
                G[w.b2 + k] += v;
            }
            for (int o = threadIdx.x; o < N * H; o += ET_THREADS) {   // dZG2 -> n3
                const int i = o / H, n = o - i * H;
                float v = 0.f;
                for (int k = 0; k < 3; ++k) v = fmaf(s.tmp[3 * i + k], P.blob[w.w2 + 4 * n + k], v);
                s.n3[o] = v * et_dsilu(sh[so.zg2 + o]);
            }
            __syncthreads();
            et_wgrad(s.n1, N, H, H, s.n3, H, H, G + w.w1, H, G + w.b1, first);
            et_bwd<HT>(s.n3, N, H, H, P.blob + w.w1, H, H, s.n4, H, false);   // dG1 -> n4
            for (int o = threadIdx.x; o < N * H; o += ET_THREADS) s.n4[o] *= et_dsilu(sh[so.zg1 + o]);   // dZG1
            __syncthreads();
            et_wgrad(s.X, N, LH, LH, s.n4, H, H, G + w.w0, H, G + w.b0, first);
            et_bwd<HT>(s.n4, N, H, H, P.blob + w.w0, H, LH, s.dX, LH, false);   // dXh [N][H+8]
            for (int o = threadIdx.x; o < N * H; o += ET_THREADS) dh[o] += s.dX[(o / H) * LH + o % H];
            for (int o = threadIdx.x; o < 3 * N; o += ET_THREADS) s.dcoord[o] += s.dX[(o / 3) * LH + H + o % 3];
            __syncthreads();
        }
        ck.tick(P, 0);
        // ---- layers, last to first
        for (int l = P.L - 1; l >= 0; --l) {
            const LayerOff w = layer_off(H, l);
            const float* sl = sv + l * so.layer;
            const float* hin = sl + so.hin;
            for (int o = threadIdx.x; o < 4 * N; o += ET_THREADS) s.coord[o] = sl[so.cin + o];
            __syncthreads();
            geometry(P, s);
            for (int e = threadIdx.x; e < E; e += ET_THREADS) {
                const float u = sl[so.u + e];
                s.cd[e] = P.use_tanh ? tanhf(u) : u;
            }
            // V1 = silu(ZV1) -> n1, vd
            for (int o = threadIdx.x; o < N * H; o += ET_THREADS) s.n1[o] = et_silu(sl[so.zv1 + o]);
            __syncthreads();
            for (int i = threadIdx.x; i < N; i += ET_THREADS) {
                float v = 0.f;
                for (int k = 0; k < 3; ++k) v = fmaf(s.dcoord[3 * i + k], s.velv[3 * i + k], v);
                s.dvd[i] = v;
            }
            // (a) coord_model: dtrans -> ddiffn (s.dX rows as [E][3] scratch), dcd
            float* ddn = s.dX;
            const float inv_deg = deg > 0 ? 1.0f / (float)deg : 0.f;
            for (int e = threadIdx.x; e < E; e += ET_THREADS) {
                const int r = e_row(e, deg);
                float dc = 0.f;
                for (int k = 0; k < 3; ++k) {
                    const float tr = s.diffn[3 * e + k] * s.cd[e];
                    const float dt = (tr >= -100.f && tr <= 100.f) ? s.dcoord[3 * r + k] * P.coords_weight * inv_deg : 0.f;
                    ddn[3 * e + k] = dt * s.cd[e];
                    dc = fmaf(dt, s.diffn[3 * e + k], dc);
                }
                s.dcd[e] = dc;
            }
            __syncthreads();
            ck.tick(P, 1);
            // (b) node_mlp: dhn = dh; N1 = silu(ZN1) -> n2; Xn = [hin, AGG] -> n3 (2H wide)
            for (int o = threadIdx.x; o < N * H; o += ET_THREADS) {
                const int i = o / H, n = o - i * H;
                s.n2[o] = et_silu(sl[so.zn1 + o]);
                s.n3[i * 2 * H + n] = hin[o];
                s.n3[i * 2 * H + H + n] = sl[so.agg + o];
            }
            __syncthreads();
            et_wgrad(s.n2, N, H, H, dh, H, H, G + w.n1, H, G + w.n1b, first);
            et_bwd<HT>(dh, N, H, H, P.blob + w.n1, H, H, s.n4, H, false);   // dN1 -> n4
            for (int o = threadIdx.x; o < N * H; o += ET_THREADS) s.n4[o] *= et_dsilu(sl[so.zn1 + o]);   // dZN1
            __syncthreads();
            et_wgrad(s.n3, N, 2 * H, 2 * H, s.n4, H, H, G + w.n0, H, G + w.n0b, first);
            // dXn = dZN1 Wn0^T -> n2 ([N][2H]); dh_in = (recurrent ? dh : 0) + dXn[:, :H]; dAGG = dXn[:, H:]
            et_bwd<HT>(s.n4, N, H, H, P.blob + w.n0, H, 2 * H, s.n2, 2 * H, false);
            float* dhin = s.n3;   // [N][H] (n3 is free again)
            for (int o = threadIdx.x; o < N * H; o += ET_THREADS) {
                const int i = o / H, n = o - i * H;
                dhin[o] = (P.recurrent ? dh[o] : 0.f) + s.n2[i * 2 * H + n];
            }
            __syncthreads();
            ck.tick(P, 2);
            // (c) coord_mlp_vel: dV1 = dvd w_v1; gw_v1, gb_v1; dZV1 -> n4; dh_in += dZV1 Wv0^T
            for (int n = threadIdx.x; n < H; n += ET_THREADS) {
                float v = 0.f;
                for (int i = 0; i < N; ++i) v = fmaf(s.dvd[i], s.n1[i * H + n], v);
                G[w.v1w + n] += v;
            }
            if (threadIdx.x == 0) {
                float v = 0.f;
                for (int i = 0; i < N; ++i) v += s.dvd[i];
                G[w.v1b] += v;
            }
            for (int o = threadIdx.x; o < N * H; o += ET_THREADS) {
                const int i = o / H, n = o - i * H;
                s.n4[o] = s.dvd[i] * P.blob[w.v1w + n] * et_dsilu(sl[so.zv1 + o]);
            }
            __syncthreads();
            et_wgrad(hin, N, H, H, s.n4, H, H, G + w.v0, H, G + w.v0b, first);
            et_bwd<HT>(s.n4, N, H, H, P.blob + w.v0, H, H, dhin, H, true);
            ck.tick(P, 3);
            // (d) coord_mlp: dU = dcd (1 - cd^2); C1 = silu(ZC1) -> A; EF = silu(ZEF) -> Bq
            for (int o = threadIdx.x; o < E * H; o += ET_THREADS) {
                s.A[o] = et_silu(sl[so.zc1 + o]);
                s.Bq[o] = et_silu(sl[so.zef + o]);
            }
            for (int e = threadIdx.x; e < E; e += ET_THREADS)
                s.dcd[e] = P.use_tanh ? s.dcd[e] * (1.0f - s.cd[e] * s.cd[e]) : s.dcd[e];   // -> dU
            __syncthreads();
            for (int n = threadIdx.x; n < H; n += ET_THREADS) {   // gw_c1 += sum_e dU_e C1_e
                float v = 0.f;
                for (int e = 0; e < E; ++e) v = fmaf(s.dcd[e], s.A[e * H + n], v);
                G[w.c1w + n] += v;
            }
            for (int o = threadIdx.x; o < E * H; o += ET_THREADS) {   // dZC1 -> Cq
                const int e = o / H, n = o - e * H;
                s.Cq[o] = s.dcd[e] * P.blob[w.c1w + n] * et_dsilu(sl[so.zc1 + o]);
            }
            __syncthreads();
            ck.tick(P, 4);
            et_wgrad(s.Bq, E, H, H, s.Cq, H, H, G + w.c0, H, G + w.c0b, first);
            ck.tick(P, 5);
            et_bwd<HT>(s.Cq, E, H, H, P.blob + w.c0, H, H, s.A, H, false);   // dEF -> A
            ck.tick(P, 6);
            // (e) dEF += dAGG[row] / deg
            for (int o = threadIdx.x; o < E * H; o += ET_THREADS) {
                const int e = o / H, n = o - e * H;
                s.A[o] += s.n2[e_row(e, deg) * 2 * H + H + n] * inv_deg;
            }
            __syncthreads();
            // (f) edge_mlp: dZEF = dEF silu'(ZEF) -> Cq; E1 = silu(ZE1) -> Bq
            for (int o = threadIdx.x; o < E * H; o += ET_THREADS) {
                s.Cq[o] = s.A[o] * et_dsilu(sl[so.zef + o]);
                s.Bq[o] = et_silu(sl[so.ze1 + o]);
            }
            __syncthreads();
            ck.tick(P, 7);
            et_wgrad(s.Bq, E, H, H, s.Cq, H, H, G + w.e1, H, G + w.e1b, first);
            ck.tick(P, 5);
            et_bwd<HT>(s.Cq, E, H, H, P.blob + w.e1, H, H, s.A, H, false);   // dE1 -> A
            ck.tick(P, 6);
            for (int o = threadIdx.x; o < E * H; o += ET_THREADS) s.A[o] *= et_dsilu(sl[so.ze1 + o]);   // dZE1
            __syncthreads();
            edge_input(P, s, hin);                                         // X (for gWe0)
            ck.tick(P, 8);
            et_wgrad(s.X, E, LX, LX, s.A, H, H, G + w.e0, H, G + w.e0b, first);
            ck.tick(P, 9);
            // dX = dZE1 We0^T, only the columns that carry gradient: [0, 2H] (h_row, h_col, radial);
            // ddn still lives in the first 3E floats of s.dX, so the product goes to s.X (X is done)
            et_bwd<HT>(s.A, E, H, H, P.blob + w.e0, H, 2 * H + 1, s.X, LX, false);
            ck.tick(P, 10);
            for (int o = threadIdx.x; o < N * H; o += ET_THREADS) {   // dh_in[row] / dh_in[col] sums
                const int i = o / H, n = o - i * H;
                float v = 0.f;
                for (int e = 0; e < E; ++e) {
                    if (e_row(e, deg) == i) v += s.X[e * LX + n];
                    if (e_col(e, deg) == i) v += s.X[e * LX + H + n];
                }
                dhin[o] += v;
            }
            // (g) geometry: ddiff = 2 dradial diff + J(diffn)^T ddiffn; dcoord[row] += ddiff, [col] -= ddiff
            float* dd = s.dX + 3 * E;   // [E][3] after ddn
            for (int e = threadIdx.x; e < E; e += ET_THREADS) {
                const float dr = s.X[e * LX + 2 * H];
                float d[3], dn[3], n[3];
                for (int k = 0; k < 3; ++k) {
                    d[k] = s.diff[3 * e + k];
                    dn[k] = ddn[3 * e + k];
                    n[k] = s.diffn[3 * e + k];
                }
                const float len = sqrtf(s.radial[e]);
                float g[3];
                if (P.norm_diff && len > 1.0f) {
                    const float nd = n[0] * dn[0] + n[1] * dn[1] + n[2] * dn[2];
                    for (int k = 0; k < 3; ++k) g[k] = (dn[k] - n[k] * nd) / len;
                } else {
                    for (int k = 0; k < 3; ++k) g[k] = dn[k];
                }
                for (int k = 0; k < 3; ++k) dd[3 * e + k] = g[k] + 2.0f * dr * d[k];
            }
            __syncthreads();
            for (int o = threadIdx.x; o < 3 * N; o += ET_THREADS) {
                const int i = o / 3, k = o - 3 * i;
                float v = 0.f;
                for (int e = 0; e < E; ++e) {
                    if (e_row(e, deg) == i) v += dd[3 * e + k];
                    if (e_col(e, deg) == i) v -= dd[3 * e + k];
                }
                s.dcoord[o] += v;
            }
            for (int o = threadIdx.x; o < N * H; o += ET_THREADS) dh[o] = dhin[o];
            __syncthreads();
            ck.tick(P, 11);
        }
        // ---- embedding: h0 = b + |vel| w[0] + mass w[1]
        for (int n = threadIdx.x; n < H; n += ET_THREADS) {
            float g0 = 0.f, g1 = 0.f, gb = 0.f;
            for (int i = 0; i < N; ++i) {
                const float vx = s.velv[3 * i], vy = s.velv[3 * i + 1], vz = s.velv[3 * i + 2];
                g0 = fmaf(sqrtf(vx * vx + vy * vy + vz * vz), dh[i * H + n], g0);
                g1 = fmaf(s.mass[i], dh[i * H + n], g1);
                gb += dh[i * H + n];
            }
            G[n] += g0;
            G[H + n] += g1;
            G[2 * H + n] += gb;
        }
        __syncthreads();
    }
    ck.tick(P, 12);
    ck.flush(P);
}

// part = 0 as a kernel rather than hipMemsetAsync: the bench captures the whole training step in a
// HIP graph, and back-to-back replays of a graph holding a memset node gave nondeterministic gradients
// (a race between one replay's memset and the previous replay's reduction); kernel nodes stay ordered
__global__ void egnn_zero_kernel(float* __restrict__ p, int64_t n, float v) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

// grad[i] = sum_g part[g][i]
__global__ void egnn_grad_reduce_kernel(const float* __restrict__ part, int G, int64_t n, float* __restrict__ grad) {
    const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = 0.f;
    for (int g = 0; g < G; ++g) v += part[(int64_t)g * n + i];
    grad[i] = v;
}

// NBX_ET_DEBUG=1: per-workgroup phase clocks of the training kernels, averaged to stderr (tuning only)
unsigned long long* et_dbg_buf() {
    static const bool on = getenv("NBX_ET_DEBUG") != nullptr;
    static unsigned long long* buf = nullptr;
    if (on && !buf && hipMalloc(&buf, sizeof(unsigned long long) * 16 * 4096) != hipSuccess) buf = nullptr;
    return on ? buf : nullptr;
}

int et_dbg_dump(const char* what, unsigned long long* dbg, int grid, hipStream_t st) {
    if (!dbg) return NBX_OK;
    std::vector<unsigned long long> h((size_t)grid * 16);
    NBX_HIP(hipStreamSynchronize(st));
    NBX_HIP(hipMemcpy(h.data(), dbg, h.size() * 8, hipMemcpyDeviceToHost));
    fprintf(stderr, "et_debug %s (avg clocks per workgroup):", what);
    for (int i = 0; i < 16; ++i) {
        double a = 0;
        for (int g = 0; g < grid; ++g) a += (double)h[(size_t)g * 16 + i];
        if (a > 0) fprintf(stderr, " [%d] %.0f", i, a / grid);
    }
    fprintf(stderr, "\n");
    return NBX_OK;
}

int64_t blob_floats(const nbx_egnn_weights* w) {
    const int64_t H = w->hidden;
    return 3 * H + w->num_layers * (8 * H * H + 16 * H + 4) + w->num_heads * (2 * H * H + 14 * H + 4);
}

int check_train(const nbx_egnn_weights* w, int64_t B, int64_t N) {
    NBX_CHECK_ARG(w && w->persist_blob, "egnn train: needs the persist blob");
    NBX_CHECK_ARG(w->hidden % 4 == 0 && w->hidden >= 4 && w->num_heads >= 1 && w->num_heads <= 2,
                  "egnn train: hidden %% 4 == 0, 1-2 heads");
    NBX_CHECK_ARG(B >= 1 && N >= 2 && N <= 8, "egnn train: 2 <= N <= 8");
    const size_t lds = train_lds_floats((int)N, w->hidden) * 4;
    if (lds > 160 * 1024) {
        nbx::set_error("egnn train: N = %lld at hidden %d needs %zu bytes of LDS", (long long)N, w->hidden, lds);
        return NBX_E_UNSUPPORTED;
    }
    return NBX_OK;
}

constexpr int TRAIN_GROUPS = 64;   // backward workgroups (partial gradient slices)

int set_lds_attr() {
    for (const void* k : {(const void*)egnn_train_fwd_kernel<0>, (const void*)egnn_train_fwd_kernel<32>,
                          (const void*)egnn_train_fwd_kernel<64>, (const void*)egnn_train_fwd_kernel<128>,
                          (const void*)egnn_train_bwd_kernel<0>, (const void*)egnn_train_bwd_kernel<32>,
                          (const void*)egnn_train_bwd_kernel<64>, (const void*)egnn_train_bwd_kernel<128>})
        NBX_LDS_160K(k);
    return NBX_OK;
}

}  // namespace

extern "C" int nbx_egnn_train_workspace_bytes(const nbx_egnn_weights* w, int64_t B, int64_t N, size_t* bytes) {
    NBX_CHECK_ARG(w && bytes && B >= 1 && N >= 2, "nbx_egnn_train_workspace_bytes: bad arguments");
    const int64_t sf = save_floats((int)N, w->hidden, w->num_layers, w->num_heads);
    const int64_t G = B < TRAIN_GROUPS ? B : TRAIN_GROUPS;
    *bytes = (size_t)(B * sf + G * blob_floats(w)) * 4;
    return NBX_OK;
}

extern "C" int nbx_egnn_train_forward(const nbx_egnn_weights* w, const float* pos, const float* vel, const float* mass,
                                      int64_t B, int64_t N, float* out, void* workspace, size_t workspace_bytes,
                                      void* stream) {
    if (int rc = check_train(w, B, N)) return rc;
    size_t need = 0;
    nbx_egnn_train_workspace_bytes(w, B, N, &need);
    NBX_CHECK_ARG(workspace && workspace_bytes >= need, "egnn train: workspace too small (%zu < %zu)", workspace_bytes, need);
    EgnnTrain p{};
    p.blob = w->persist_blob; p.L = w->num_layers; p.N = (int)N; p.heads = w->num_heads; p.recurrent = w->recurrent;
    p.norm_diff = w->norm_diff; p.use_tanh = w->use_tanh; p.H = w->hidden; p.coords_weight = w->coords_weight;
    p.pos = pos; p.vel = vel; p.mass = mass; p.B = B;
    p.save = static_cast<float*>(workspace);
    p.save_floats = save_floats((int)N, w->hidden, w->num_layers, w->num_heads);
    p.out = out;
    p.dbg = et_dbg_buf();
    const size_t lds = train_lds_floats((int)N, w->hidden) * 4;
    if (int rc = set_lds_attr()) return rc;
    switch (w->hidden) {
        case 32: hipLaunchKernelGGL(egnn_train_fwd_kernel<32>, dim3((unsigned)B), dim3(ET_THREADS), lds, (hipStream_t)stream, p); break;
        case 64: hipLaunchKernelGGL(egnn_train_fwd_kernel<64>, dim3((unsigned)B), dim3(ET_THREADS), lds, (hipStream_t)stream, p); break;
        case 128: hipLaunchKernelGGL(egnn_train_fwd_kernel<128>, dim3((unsigned)B), dim3(ET_THREADS), lds, (hipStream_t)stream, p); break;
        default: hipLaunchKernelGGL(egnn_train_fwd_kernel<0>, dim3((unsigned)B), dim3(ET_THREADS), lds, (hipStream_t)stream, p);
    }
    NBX_HIP(hipGetLastError());
    return et_dbg_dump("forward", p.dbg, (int)B, (hipStream_t)stream);
}

extern "C" int nbx_egnn_train_backward(const nbx_egnn_weights* w, const float* pos, const float* vel,
                                       const float* mass, int64_t B, int64_t N, const float* grad_out, float* grad_blob,
                                       void* workspace, size_t workspace_bytes, void* stream) {
    if (int rc = check_train(w, B, N)) return rc;
    size_t need = 0;
    nbx_egnn_train_workspace_bytes(w, B, N, &need);
    NBX_CHECK_ARG(workspace && workspace_bytes >= need && grad_out && grad_blob,
                  "egnn train backward: workspace too small or null gradient buffers");
    hipStream_t st = (hipStream_t)stream;
    EgnnTrain p{};
    p.blob = w->persist_blob; p.L = w->num_layers; p.N = (int)N; p.heads = w->num_heads; p.recurrent = w->recurrent;
    p.norm_diff = w->norm_diff; p.use_tanh = w->use_tanh; p.H = w->hidden; p.coords_weight = w->coords_weight;
    p.pos = pos; p.vel = vel; p.mass = mass; p.B = B;
    p.save = static_cast<float*>(workspace);
    p.save_floats = save_floats((int)N, w->hidden, w->num_layers, w->num_heads);
    p.dout = grad_out;
    p.blob_floats = blob_floats(w);
    p.gpart = p.save + B * p.save_floats;
    const int G = (int)(B < TRAIN_GROUPS ? B : TRAIN_GROUPS);
    p.dbg = et_dbg_buf();
    // NBX_ET_MEMSET=1: the old hipMemsetAsync zeroing (diagnosis of the graph-replay race only,
    // tools/egnn_graph_dump.py)
    static const bool use_memset = getenv("NBX_ET_MEMSET") && getenv("NBX_ET_MEMSET")[0] == '1';
    if (use_memset) {
        NBX_HIP(hipMemsetAsync(p.gpart, 0, sizeof(float) * (size_t)G * p.blob_floats, st));
    } else {
        hipLaunchKernelGGL(egnn_zero_kernel, dim3(4096), dim3(256), 0, st, p.gpart, (int64_t)G * p.blob_floats, 0.f);
    }
    const size_t lds = train_lds_floats((int)N, w->hidden) * 4;
    if (int rc = set_lds_attr()) return rc;
    switch (w->hidden) {
        case 32: hipLaunchKernelGGL(egnn_train_bwd_kernel<32>, dim3((unsigned)G), dim3(ET_THREADS), lds, st, p); break;
        case 64: hipLaunchKernelGGL(egnn_train_bwd_kernel<64>, dim3((unsigned)G), dim3(ET_THREADS), lds, st, p); break;
        case 128: hipLaunchKernelGGL(egnn_train_bwd_kernel<128>, dim3((unsigned)G), dim3(ET_THREADS), lds, st, p); break;
        default: hipLaunchKernelGGL(egnn_train_bwd_kernel<0>, dim3((unsigned)G), dim3(ET_THREADS), lds, st, p);
    }
    NBX_HIP(hipGetLastError());
    if (int rc = et_dbg_dump("backward", p.dbg, G, st)) return rc;
    hipLaunchKernelGGL(egnn_grad_reduce_kernel, dim3((unsigned)((p.blob_floats + 255) / 256)), dim3(256), 0, st, p.gpart,
                       G, p.blob_floats, grad_blob);
    NBX_HIP(hipGetLastError());
    return NBX_OK;
}
