// update_layer_1, split form (segmented input, mul = 96, bf16x3): the vector GEMM of all M output
// channels in one kernel, the scalar GEMM + gate in tp16 (EPI TP_GATE_VRAW, NV = 0).
//
// Why: in the combined tp16 kernel a wave owns one 16-channel chunk, so every 1o A element it splits
// into bf16x3 parts (~5.5 VALU) feeds a single 16-column output tile (6 MFMAs per 32-deep K item):
// the kernel is VALU-issue bound (2 600 VALU against 288 MFMAs per wave, PMC r02).  Here a wave owns a
// 16-row tile of the stacked 1o rows [3 planes x V nodes] and all 96 output columns, so a split A
// element feeds 6 tiles (36 MFMAs per item), and the scalar kernel keeps only the 0e items.
//
//   v_raw[k][n][c] = sum_j W_v[c][j] A[k][n][j],  A = [s_x . x_v[:, k] | s_m . a_v[:, k]]   (K = 2M)
//
// s_x: the pending feature BatchNorm's 1o scale (xcoef[M + j], identity at layer 0); s_m: the
// message BatchNorm's 1o scale, finalised here from its sums (mbn) -- block 0 also finalises every
// other message-BN coefficient into mbn.coef_out and applies the running-statistics update, so the
// scalar kernel reads plain coefficients (mcoef) -- or read from mcoef when the sums are not in use.
// Weights: the vector sub-tile of each 16-channel chunk of the upd1 bf16x3 image (include/nbx.h
// "bf16x3 images"), staged by LDS-DMA as [chunk][kc][part][lane] bf16x8.
#pragma once
#include "tp_fused.h"

namespace nbx {

struct UpdVecProb {
    const float* xv;      // x_v plane 0 ([3][V][M], planes V*M apart; pre-BN values)
    const float* av;      // a_v plane 0 (raw aggregated messages)
    const float* img;     // upd1 bf16x3 image: chunk c at img + c * img_stride
    int img_stride;       // floats per chunk image
    int vec_off;          // floats from a chunk image's start to its vector sub-tile
    const float* xcoef;   // [sc_s | sc_v | sh] of the pending feature BN, or null (identity)
    const float* mcoef;   // message BN coefficients when mbn.sums is null
    BnSrc mbn;            // message BN finalised here (sums non-null)
    float* out;           // v_raw [3][V][M]
    int64_t V;
    int M;
};

constexpr int UV_WAVES = 4, UV_CHUNKS = 6, UV_KC = 6;   // M = 96: 6 chunks of 16 channels, K = 192
constexpr int UV_VEC_FLOATS = UV_KC * 768;              // one chunk's vector sub-tile (x3): 6 x 3 KiB
constexpr int UV_LDS_FLOATS = UV_CHUNKS * UV_VEC_FLOATS + 2 * 96;   // images + the 2M scale table

__global__ __launch_bounds__(64 * UV_WAVES, 1) void upd_vec_kernel(const UpdVecProb P) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int M = 96;
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63, c16 = lane & 15, qd = lane >> 4;
    const int64_t R = 3 * P.V;
    const int64_t tile = (int64_t)blockIdx.x * UV_WAVES + wave;
    const int64_t row = tile * 16 + c16;
    const bool rok = row < R;
    const int64_t plane = rok ? row / P.V : 0, node = rok ? row - plane * P.V : 0;

    // A prefetch: all 6 K items of this lane's row (8 consecutive k per item), bounds-checked
    // buffer loads (invalid rows read zeros); issued before the weight staging
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)P.xv, (short)0, 0x7FFFFFF0, 0x00020000);
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)P.av, (short)0, 0x7FFFFFF0, 0x00020000);
    float4 a[UV_KC][2];
    {
        const uint32_t base = rok ? (uint32_t)(((uint64_t)plane * P.V * M + (uint64_t)node * M) * 4) : 0x7FFFFFF0u;
#pragma unroll
        for (int kc = 0; kc < UV_KC; ++kc) {
            const uint32_t off = rok ? base + (uint32_t)(((kc % 3) * 32 + 8 * qd) * 4) : base;
            const __amdgpu_buffer_rsrc_t& rs = kc < 3 ? rx : ra;
            a[kc][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
            a[kc][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, rok ? off + 16 : off, 0, 0));
        }
    }
    // stage the 6 vector sub-tiles (LDS-DMA, 18 KiB each)
#pragma unroll
    for (int c = 0; c < UV_CHUNKS; ++c)
        tp_dma_image<UV_WAVES>(P.img + (size_t)c * P.img_stride + P.vec_off, lds + c * UV_VEC_FLOATS, UV_VEC_FLOATS);
    // 1o scales: j < M from the feature BN (x_v), j >= M from the message BN (a_v); block 0 finalises
    // every message-BN coefficient (running statistics, coef_out) once
    float* sc = lds + UV_CHUNKS * UV_VEC_FLOATS;
    if (t < M) {
        sc[t] = P.xcoef ? P.xcoef[M + t] : 1.0f;
        if (P.mbn.sums) {
            const bool own = blockIdx.x == 0;
            sc[M + t] = bn_coef(P.mbn, M, 1, t, own);
            if (own) {
                (void)bn_coef(P.mbn, M, 0, t, true);
                (void)bn_coef(P.mbn, M, 2, t, true);
            }
        } else {
            sc[M + t] = P.mcoef[M + t];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    floatx4 acc[UV_CHUNKS];
#pragma unroll
    for (int c = 0; c < UV_CHUNKS; ++c) acc[c] = floatx4{0.f, 0.f, 0.f, 0.f};
    constexpr int TA[6] = {2, 1, 0, 1, 0, 0}, TB[6] = {0, 1, 2, 0, 1, 0};
    const bf16x8* img = reinterpret_cast<const bf16x8*>(lds);
#pragma unroll
    for (int kc = 0; kc < UV_KC; ++kc) {
        // this item's k = 32 (kc % 3) + 8 qd + e of segment kc / 3 (x_v, then a_v)
        const float* s = sc + (kc / 3) * M + (kc % 3) * 32 + 8 * qd;
        const float4 s0 = *reinterpret_cast<const float4*>(s);
        const float4 s1 = *reinterpret_cast<const float4*>(s + 4);
        const float4 v0 = make_float4(a[kc][0].x * s0.x, a[kc][0].y * s0.y, a[kc][0].z * s0.z, a[kc][0].w * s0.w);
        const float4 v1 = make_float4(a[kc][1].x * s1.x, a[kc][1].y * s1.y, a[kc][1].z * s1.z, a[kc][1].w * s1.w);
        bf16x8 ax[3];
        tp_split3(v0, v1, ax[0], ax[1], ax[2]);
#pragma unroll
        for (int c = 0; c < UV_CHUNKS; ++c) {
            bf16x8 bx[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) bx[p] = img[((c * UV_KC + kc) * 3 + p) * 64 + lane];
#pragma unroll
            for (int tt = 0; tt < 6; ++tt)
                acc[c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax[TA[tt]], bx[TB[tt]], acc[c], 0, 0, 0);
        }
    }
    // C register j -> row 4 qd + j of the tile, column c16 of chunk c
    asm volatile("s_nop 0" ::: "memory");
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t r = tile * 16 + 4 * qd + j;
        if (r >= R) continue;
        const int64_t pl = r / P.V, n = r - pl * P.V;
        float* o = P.out + (pl * P.V + n) * M + c16;
#pragma unroll
        for (int c = 0; c < UV_CHUNKS; ++c) o[16 * c] = acc[c][j];
    }
}

inline int upd_vec_launch(const UpdVecProb& p, hipStream_t st) {
    if (p.M != 96) {
        set_error("upd_vec: mul must be 96");
        return NBX_E_UNSUPPORTED;
    }
    if ((double)3 * p.V * p.M * 4.0 >= 2147483632.0) {
        set_error("upd_vec: input spans >= 2 GiB (32-bit buffer offsets)");
        return NBX_E_UNSUPPORTED;
    }
    static bool attr_set = false;
    if (!attr_set) {
        NBX_HIP(hipFuncSetAttribute((const void*)upd_vec_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    160 * 1024));
        attr_set = true;
    }
    const int64_t tiles = (3 * p.V + 15) / 16;
    const unsigned blocks = (unsigned)((tiles + UV_WAVES - 1) / UV_WAVES);
    NBX_TIMED_LAUNCH(upd_vec_kernel, dim3(blocks), dim3(64 * UV_WAVES), (size_t)UV_LDS_FLOATS * 4, st, p);
    NBX_HIP(hipGetLastError());
    return NBX_OK;
}

}  // namespace nbx
